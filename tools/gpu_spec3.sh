# GPU tests on the default build, then same-box spectrum/chain timing of the
# library variants named in $1 (default: stream-kernel build vs default).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
LIBS=${1:-"libdspcore_stream.so libdspcore.so"}
OUT=gpurun_out/spec3; mkdir -p $OUT
echo "== gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest.log | head -30; exit $rc; }
echo "== timing"
bash tools/gpu_specab.sh spec3 "$LIBS" > $OUT/timing.log 2>&1 || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/spec3/timing.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["tag"], d["B"], d["step_ms"], d["kernels_ms"])
PY
python tools/tile_ab.py --compare c3_libdspcore_prev c3_libdspcore | tee $OUT/compare.txt
