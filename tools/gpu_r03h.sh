set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_h; mkdir -p $OUT
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; exit $rc; }
echo "== lds broadcast ubench"
timeout -k 10 60 ./tools/ubench_lds_bcast | tee $OUT/ubench_lds_bcast.txt
