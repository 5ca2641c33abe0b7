# Same-box A/B of library builds on configs 3/4 and 5 (tools/tile_ab.py):
#   bash tools/gpu_ab_r04.sh OUTDIR lib:flushed ...   (flushed = 1 for builds before ABI 2.1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for pass in 1 2; do
for spec in "$@"; do
  lib=${spec%%:*}; fl=${spec#*:}; [ "$fl" = 1 ] || fl=
  for cfg in c3 c5; do
    ch="4096 32768"; [ $cfg = c5 ] && ch=8192
    DSP_AB_FLUSHED=$fl DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${lib%.so}_p$pass" --config $cfg --channels $ch --steps 20 2>&1 | grep -v amdgpu.ids >> $OUT/ab.log || exit 1
  done
done
done
cat $OUT/ab.log
