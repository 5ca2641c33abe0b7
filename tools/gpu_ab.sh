# GPU parity tests + smoke + bench line, then a same-box A/B of library builds
# on the single-pass chain (configs 3/4 geometry and config 5) -> gpurun_out/$TAG/.
#   bash tools/gpu_ab.sh TAG "lib1.so lib2.so ..." [bench configs, default c4; none skips]
set -o pipefail
TAG=$1; LIBS=$2; shift 2
CFGS=${*:-c4}
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh "$TAG" $CFGS || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for cfg in c3 c5; do
  CH="4096 32768"; [ $cfg = c5 ] && CH="8192"
  for lib in $LIBS; do
    DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${cfg}_${lib%.so}" --config $cfg --channels $CH 2>&1 | grep -v amdgpu.ids | tee -a "$OUT/ab.jsonl" || exit 1
  done
done
first=${LIBS%% *}; first=${first%.so}
for lib in $LIBS; do
  python tools/tile_ab.py --compare "c3_$first" "c3_${lib%.so}" | tee -a "$OUT/ab_compare.txt"
  python tools/tile_ab.py --compare "c5_$first" "c5_${lib%.so}" | tee -a "$OUT/ab_compare.txt"
done
