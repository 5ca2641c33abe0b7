set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; rm -rf $OUT; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for pass in 1 2; do for lib in "$@"; do
  DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${lib%.so}_p$pass" --config c5 --channels 8192 --steps 20 --path 3 2>&1 | grep -v amdgpu.ids >> $OUT/ab.log || exit 1
done; done
grep '^{' $OUT/ab.log | cut -c1-200
