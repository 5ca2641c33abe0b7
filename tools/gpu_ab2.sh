# A/B of library builds with fusion on/off: bash tools/gpu_ab2.sh lib1 lib2 ...
# (CHAIN_LM="2,1" for the L/M = 2/1 geometry; libraries as in tools/build_variants.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  DSPCORE_LIB="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib/$lib" timeout -k 10 120 python tools/fused_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
done
