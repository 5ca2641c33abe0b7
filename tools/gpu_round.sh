# Round measurement: GPU parity tests, smoke, bench lines (config 4 default and
# config 5), rocprofv3 kernel stats of the same bench commands, PMC passes
# (HBM traffic + SQ counters, run first so the bench lines cite them) -> gpurun_out/$TAG/.
#   bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
rm -rf "$OUT"; mkdir -p "$OUT"
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
# PMC passes first, so that the bench lines below cite this run's traffic:
# pmc_traffic.json is rewritten on the box (and copied back under gpurun_out/).
cd "$GRAFT_REPO_ROOT"
for c in c4 c5 c3; do
  case $c in c4) wl=config4; ch=32768;; c5) wl=config5; ch=8192;; c3) wl=config3; ch=4096;; esac
  bash tools/pmc_chain.sh "$TAG/pmc_$c" 3 $c > "$OUT/pmc_$c.log" 2>&1 || { tail -20 "$OUT/pmc_$c.log"; exit 1; }
  python tools/pmc_parse.py "$OUT/pmc_$c/pmc" --write $wl $ch "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/kernels_once.py (profiles/${TAG}_${c}_pmc_summary.txt)" > /dev/null || exit 1
  grep -E "^==|traffic" "$OUT/pmc_$c/pmc_summary.txt"
done
cp pmc_traffic.json "$OUT/pmc_traffic.json"
for c in c4 c5; do
  echo "== bench $c"
  extra=""; [ $c = c5 ] && extra="--no-extras"
  timeout -k 10 600 python bench.py --config $c $extra > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -20 "$OUT/bench_$c.err"; exit 1; }
  cut -c1-300 "$OUT/bench_$c.json"
done
cd /tmp && export TMPDIR=/tmp
for c in c4 c5; do
  echo "== rocprof stats $c"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $c --steps 20 --warmup 5 --cpu-per-proc 0 --no-config3 > "$OUT/prof_$c.log" 2>&1 || { tail -20 "$OUT/prof_$c.log"; exit 1; }
  find "$OUT/prof_$c" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_$c.csv" \;
  cut -d, -f1-4 "$OUT/kernel_stats_$c.csv" | head -4 | cut -c1-200
  grep '^{' "$OUT/prof_$c.log" | cut -c1-200
done
echo done
