# Pipelined-cascade bring-up: GPU parity, then A/B against the serial cascade
# (libdspcore_ser.so) with fusion on and off, both fused geometries.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_pipe.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh libdspcore.so libdspcore_ser.so libdspcore_e3.so || exit 1
CHAIN_LM=2,1 bash tools/gpu_ab2.sh libdspcore.so libdspcore_ser.so || exit 1
