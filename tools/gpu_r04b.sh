# Round 4: the non-finite tests, the GPU suite, then a same-box A/B (tile_ab.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04b}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_nonfinite.py -x -v --timeout 300 --timeout-method thread > $OUT/nonfinite.log 2>&1 || { tail -40 $OUT/nonfinite.log; exit 1; }
tail -3 $OUT/nonfinite.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_nonfinite.py > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
bash tools/gpu_ab_r04.sh ${1:-r04b} libdspcore_head.so:1 libdspcore.so:0 > /dev/null || exit 1
python3 - $OUT/ab.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    try:
        d = json.loads(l)
    except ValueError:
        continue
    print(d["tag"], d["B"], d["handoff_ok"], d["step_ms"], d["kernels_ms"])
PY
