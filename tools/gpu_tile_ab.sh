# A/B of the single-pass chain kernel: baseline build vs the in-tree build
# (and R = 1), then the GPU parity tests on the in-tree build.
#   bash tools/gpu_tile_ab.sh BASELIB [channels...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
BASE=${1:-libdspcore_base.so}; shift
CH=${*:-4096 32768}
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
rm -rf gpurun_out/ab
DSPCORE_LIB="$L/$BASE" timeout -k 10 300 python tools/tile_ab.py --tag base --channels $CH 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python tools/tile_ab.py --tag new --channels $CH 2>&1 | grep -v amdgpu.ids || exit 1
DSP_CHAIN_RUN=1 timeout -k 10 300 python tools/tile_ab.py --tag new1 --channels 4096 2>&1 | grep -v amdgpu.ids || exit 1
python tools/tile_ab.py --compare base new && python tools/tile_ab.py --compare new new1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/ab/pytest.log; exit $rc
