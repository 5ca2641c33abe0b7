# Same-box A/B of library builds on config 4 (32768 channels) and config 3
# (4096), two alternating passes:  bash tools/gpu_ab_c4.sh OUT lib ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; rm -rf $OUT; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for pass in 1 2; do
  for lib in "$@"; do
    DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${lib%.so}_p$pass" \
      --config c3 --channels 32768 4096 --steps 20 2>&1 | grep -v amdgpu.ids >> $OUT/ab.log || exit 1
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
