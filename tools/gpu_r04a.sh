# Round 4: non-finite tests, the GPU suite, then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04a; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_nonfinite.py -v --timeout 300 --timeout-method thread > $OUT/nonfinite.log 2>&1
rc=$?; tail -15 $OUT/nonfinite.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_nonfinite.py > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cut -c1-600 $OUT/bench.json
exit $rc
