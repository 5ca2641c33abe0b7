set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_f; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in libdspcore.so libdspcore_dstore.so libdspcore.so libdspcore_dstore.so; do
  for cfg in c3 c5; do
    CH="4096 32768"; [ $cfg = c5 ] && CH="8192"
    DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${cfg}_${lib%.so}" --config $cfg --channels $CH 2>&1 | grep -v amdgpu.ids | tee -a $OUT/dstore.jsonl || exit 1
  done
done
python tools/tile_ab.py --compare c3_libdspcore c3_libdspcore_dstore | tee -a $OUT/dstore.jsonl
python tools/tile_ab.py --compare c5_libdspcore c5_libdspcore_dstore | tee -a $OUT/dstore.jsonl
for lib in BASE NOSRC NOP1 NOSCAN NOP2 NOYST NOZST BASE; do
  DSPCORE_LIB="$L/libdspcore_$lib.so" timeout -k 10 300 python tools/tile_ab.py --tag "abl_$lib" --config c3 --channels 4096 32768 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ablation.jsonl || exit 1
done
