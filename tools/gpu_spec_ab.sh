# Spectrum-kernel variants: parity tests, then same-box timing (tools/tile_ab.py).
#   bash tools/gpu_spec_ab.sh OUT lib ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$1; shift; rm -rf gpurun_out/$OUT; mkdir -p gpurun_out/$OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in "$@"; do
  DSPCORE_LIB="$L/$lib" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spectrum or fft or chain" --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest_${lib%.so}.log 2>&1 || { echo "FAIL $lib"; tail -20 gpurun_out/$OUT/pytest_${lib%.so}.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/$OUT/pytest_${lib%.so}.log)"
done
bash tools/gpu_ab_only.sh $OUT $(for l in "$@"; do echo "$l:0"; done)
