# Chain-kernel timing for several library builds on one workload, same box:
#   bash tools/gpu_libs_cfg.sh CONFIG "channels..." lib1.so lib2.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
CFG=$1; CH=$2; shift 2
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in "$@"; do
  DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --config "$CFG" --tag "${lib%.so}" --channels $CH 2>&1 | grep -v amdgpu.ids || exit 1
done
python tools/tile_ab.py --compare "${1%.so}" "${2%.so}"
