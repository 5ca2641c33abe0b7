# k_chain_g5 tap-block variants vs k_chain_gct, same box (config 5, 8192 channels).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/g5b; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in libdspcore_gct.so libdspcore.so libdspcore_tb4.so libdspcore_tb8.so libdspcore_gct.so libdspcore_tb8.so; do
  DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "c5_${lib%.so}" --config c5 --channels 8192 2>&1 | grep -v amdgpu.ids | tee -a $OUT/timing.jsonl || exit 1
done
python tools/tile_ab.py --compare c5_libdspcore_gct c5_libdspcore_tb8 | tee $OUT/compare.txt
