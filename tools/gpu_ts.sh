# Tile-width experiment for the fused IIR kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in libdspcore.so libdspcore_ts64.so libdspcore_ts128.so; do
  DSPCORE_LIB="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib/$lib" timeout -k 10 120 python tools/iir_ts.py 2>&1 | grep -v amdgpu.ids || exit 1
done
