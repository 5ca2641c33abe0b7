# Fused chain bring-up: new parity tests first, then the GPU suite, then bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused or config3_full" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_fused.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));print(d['value'],d['ms_per_step'],d['kernels_ms'],d['roofline'])"
timeout -k 10 300 python bench.py --cpu-sample 0 --config c5 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail -20 gpurun_out/bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c5.json'));print(d['value'],d['ms_per_step'],d['kernels_ms'])"
