# Matrix-core SRC variant: chain tests against it, then same-box timing vs the base build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/mf; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
echo "== chain tests with libdspcore_mf.so"
DSPCORE_LIB=$L/libdspcore_mf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain_contract.py -m gpu -k "chain or app_call or shard" -v --timeout 200 --timeout-method thread > $OUT/pytest_mf.log 2>&1
rc=$?; tail -3 $OUT/pytest_mf.log; grep -E "FAILED|^E " $OUT/pytest_mf.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== timing"
bash tools/gpu_libs.sh "4096 32768" libdspcore.so libdspcore_mf.so libdspcore.so libdspcore_mf.so 2>&1 | tee $OUT/timing.jsonl
python tools/tile_ab.py --compare libdspcore libdspcore_mf | tee $OUT/compare.txt
