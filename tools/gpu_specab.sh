# Same-box A/B of library builds on the spectrum kernel (and chain) at configs 3/4/5.
#   bash tools/gpu_specab.sh TAG "lib1.so lib2.so ..."
set -o pipefail
TAG=$1; LIBS=$2
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in $LIBS; do
  for cfg in c3 c5; do
    CH="4096 32768"; [ $cfg = c5 ] && CH="8192"
    DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${cfg}_${lib%.so}" --config $cfg --channels $CH 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.jsonl || exit 1
  done
done
