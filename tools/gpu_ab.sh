# A/B of library builds (DSPCORE_LIB) on the config-3 chain: bash tools/gpu_ab.sh lib1 lib2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  DSPCORE_LIB="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib/$lib" timeout -k 10 120 python tools/chain_kernels.py 2>&1 | grep -v amdgpu.ids || exit 1
done
