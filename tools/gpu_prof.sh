# rocprofv3 kernel stats of one bench run plus the PMC passes of
# tools/pmc_chain.sh -> gpurun_out/$TAG/.
#   bash tools/gpu_prof.sh TAG [config] [channels]
set -o pipefail
TAG=${1:-prof}
CFG=${2:-c3}
CH=${3:-}
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
ARGS="--config $CFG --cpu-per-proc 0 --no-config3"
[ -n "$CH" ] && ARGS="$ARGS --channels $CH"
echo "== rocprof stats ($ARGS)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-8 "$OUT/kernel_stats.csv" | grep -v "at::native" | head -8
grep '^{' "$OUT/prof.log" | head -1 | cut -c1-600
echo "== pmc"
bash "$GRAFT_REPO_ROOT/tools/pmc_chain.sh" "$TAG" 3 "$CFG" $CH | grep -E "^==|traffic|VALU |WAVE_CYCLES|BUSY|GUI"
