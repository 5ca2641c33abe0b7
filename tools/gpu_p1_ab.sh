# The L3/M2 single-pass kernel with a float64 pass 1 (lib/libdspcore_p1.so)
# against the shipped float32 pass 1: the +-15 dB precision test on both (max
# |z - oracle| per eq.npz case, and the two-launch chain's beside it), then
# config 4 / config 3 timing, two alternations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for v in "" _p1; do
  echo "== precision$v"
  DSPCORE_LIB=$L/libdspcore$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chain_contract.py -q -s -k "extreme_gains and 48000" --timeout 120 --timeout-method thread 2>&1 | grep -E "max\|z|passed|failed" || exit 1
done
for rep in 1 2; do
  for v in "" _p1; do
    DSPCORE_LIB=$L/libdspcore$v.so timeout -k 10 300 python tools/tile_ab.py --tag "p1ab${v}_$rep" --channels 32768 4096 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
