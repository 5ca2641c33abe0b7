# Iteration pass: GPU parity tests, IIR variants, quick bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/iir_variants.py > gpurun_out/iir_variants.txt 2>&1 || { tail -20 gpurun_out/iir_variants.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/iir_variants.txt
timeout -k 10 300 python bench.py --cpu-sample 0 "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));print(d['value'],d['ms_per_step'],d['kernels_ms'],d['chain_roofline']['frac'])"
