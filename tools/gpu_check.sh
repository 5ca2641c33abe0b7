# GPU parity tests, smoke and bench lines -> gpurun_out/$TAG/.
#   bash tools/gpu_check.sh TAG [bench configs...]   (default: c4; "none" skips)
set -o pipefail
TAG=${1:-check}
shift
CFGS=${*:-c4}
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
rm -rf "$OUT"; mkdir -p "$OUT"
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" "$OUT/pytest_gpu.log" | tail -3; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
for c in $CFGS; do
  [ "$c" = none ] && continue
  echo "== bench $c"
  timeout -k 10 600 python bench.py --config $c > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -20 "$OUT/bench_$c.err"; exit 1; }
  cut -c1-400 "$OUT/bench_$c.json"
  python -c "import json,sys; d=json.load(open('$OUT/bench_$c.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'kernels', d['kernels_ms'], 'frac', d['roofline']['frac'], 'chain', d['chain_roofline']['frac'], 'cfg3', (d.get('config3') or {}).get('ms_per_step'), (d.get('config3') or {}).get('kernels_ms'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), (d.get('cpu_baseline') or {}).get('cores'))"
done
