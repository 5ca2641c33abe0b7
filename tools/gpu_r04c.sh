# Round 4: the whole GPU suite, then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04c}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('$OUT/bench.json').readline())
print(d['value'], d['ms_per_step'], d['roofline']['mean_ms'], d['roofline']['frac'], d['kernels_ms'])
print('c3', d['config3']['value'], d['config3']['kernels_ms']); print('c5', d['config5']['value'], d['config5']['kernels_ms'])"
