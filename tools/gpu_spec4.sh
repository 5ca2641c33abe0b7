# Wave-kernel prefetch variants (PF 2 = L2 touch, 0 = none, 1 = registers) vs the default build: spectrum tests on the PF-2 build, then same-box timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/spec4
# the GPU tests on the PF=2 wave build (the default build's were run in r03_final4)
DSPCORE_LIB=$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib/libdspcore_wave.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "spectrum or stft or chain_config3" --timeout 200 --timeout-method thread > gpurun_out/spec4/pytest_wave.log 2>&1; rc=$?; tail -2 gpurun_out/spec4/pytest_wave.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_specab.sh spec4 "libdspcore.so libdspcore_wave.so libdspcore_wave0.so libdspcore_wave1.so libdspcore.so libdspcore_wave.so" > gpurun_out/spec4/timing.log 2>&1 || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/spec4/timing.log"):
    if l.startswith("{"):
        d = json.loads(l); print(d["tag"], d["B"], d["step_ms"], d["kernels_ms"])
PY
