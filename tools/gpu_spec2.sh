# GPU tests on the default build, then same-box spectrum/chain timing of
# libdspcore_prev.so (round-3 spectrum kernel), libdspcore_mcr.so (correctly
# rounded |X|) and libdspcore.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/spec2; mkdir -p $OUT
echo "== gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest.log | head -30; exit $rc; }
echo "== timing"
bash tools/gpu_specab.sh spec2 "libdspcore_prev.so libdspcore_mcr.so libdspcore.so libdspcore_prev.so libdspcore.so" > $OUT/timing.log 2>&1 || exit 1
python tools/tile_ab.py --compare c3_libdspcore_prev c3_libdspcore | tee $OUT/compare.txt
