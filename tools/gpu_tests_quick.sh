# GPU parity tests then a quick bench (no CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-sample 0 "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));print(d['value'],d['ms_per_step'],d['kernels_ms'],d['chain_roofline'],d['roofline'])"
