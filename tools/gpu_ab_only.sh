# Same-box A/B only: bash tools/gpu_ab_only.sh OUT lib:flushed ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$1; rm -rf gpurun_out/$OUT
bash tools/gpu_ab_r04.sh "$@" > /dev/null || { tail -20 gpurun_out/$OUT/ab.log; exit 1; }
python3 - gpurun_out/$OUT/ab.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    try:
        d = json.loads(l)
    except ValueError:
        continue
    print(d["tag"], d["B"], d["handoff_ok"], d["step_ms"], d["kernels_ms"])
PY
