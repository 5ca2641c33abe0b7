# Whole GPU suite on the in-tree library, then a same-box A/B of library
# builds on configs 4/3 (32768 / 4096 channels) and 5 (8192), two passes.
#   bash tools/gpu_suite_ab.sh OUT lib ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for pass in 1 2; do
  for lib in "$@"; do
    DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${lib%.so}_p$pass" \
      --config c3 --channels 32768 4096 --steps 20 2>&1 | grep -v amdgpu.ids >> $OUT/ab.log || exit 1
    DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${lib%.so}_p$pass" \
      --config c5 --channels 8192 --steps 20 2>&1 | grep -v amdgpu.ids >> $OUT/ab.log || exit 1
  done
done
python3 - $OUT/ab.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    try:
        d = json.loads(l)
    except ValueError:
        continue
    print(d["tag"], d["B"], d["handoff_ok"], d["step_ms"], d["kernels_ms"])
PY
