# Chain-kernel timing for several library builds (DSPCORE_LIB), same box:
#   bash tools/gpu_libs.sh "4096 32768" lib1.so lib2.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
CH=$1; shift
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in "$@"; do
  DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${lib%.so}" --channels $CH 2>&1 | grep -v amdgpu.ids || exit 1
done
