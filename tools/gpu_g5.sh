# Config-5 class-uniform kernel (k_chain_g5): chain tests, then same-box timing vs k_chain_gct (libdspcore_gct.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/g5; mkdir -p $OUT
echo "== chain tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain_contract.py -m gpu -k "chain or app_call or shard or extreme or handoff" -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest.log | head -30; exit $rc; }
echo "== timing"
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in libdspcore_gct.so libdspcore.so libdspcore_gct.so libdspcore.so; do
  DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "c5_${lib%.so}" --config c5 --channels 8192 1024 2>&1 | grep -v amdgpu.ids | tee -a $OUT/timing.jsonl || exit 1
done
python tools/tile_ab.py --compare c5_libdspcore_gct c5_libdspcore | tee $OUT/compare.txt
