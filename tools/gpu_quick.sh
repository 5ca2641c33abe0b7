# Quick measurement pass: microbenchmarks + bench kernels (no tests).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -x tools/ubench_fp64 ]; then timeout -k 10 120 tools/ubench_fp64 > gpurun_out/ubench_fp64.txt 2>&1 || exit 1; cat gpurun_out/ubench_fp64.txt; fi
timeout -k 10 300 python bench.py --cpu-sample 0 "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));print(d['value'],d['ms_per_step'],d['kernels_ms'],d['chain_roofline'])"
