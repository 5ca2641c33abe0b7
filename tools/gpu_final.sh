# Round measurement on one box: tests, smoke, bench (config 3 with CPU baseline,
# config 5), rocprofv3 kernel stats of the config-3 bench -> gpurun_out/$TAG.
set -o pipefail
TAG=${1:-r01}
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
rm -rf "$OUT"; mkdir -p "$OUT"
echo "== pytest gpu"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "== bench c3"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "== bench c5"
timeout -k 10 600 python bench.py --config c5 --cpu-sample 0 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { tail -20 "$OUT/bench_c5.err"; exit 1; }
cat "$OUT/bench_c5.json"
echo "== rocprof stats"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --cpu-sample 0 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -6
