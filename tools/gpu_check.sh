set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== pytest gpu" 
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -3 || exit 1
echo "== bench"
timeout -k 10 600 python bench.py > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err || { tail -20 gpurun_out/bench_r01.err; exit 1; }
cat gpurun_out/bench_r01.json
echo "== rocprof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r01" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --cpu-sample 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_r01.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_r01.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/prof_r01" -name "*stats*" | head
