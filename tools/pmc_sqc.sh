# Scalar-cache counters of the chain kernels -> gpurun_out/$TAG/sqc
set -o pipefail
TAG=${1:-sqc}
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT/sqc"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group -d "$OUT/sqc/p$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/kernels_once.py" 3 > "$OUT/sqc/p$i.log" 2>&1 || { tail -20 "$OUT/sqc/p$i.log"; exit 1; }
done <<'GROUPS'
SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_TC_DATA_READ_REQ SQC_TC_STALL SQ_INSTS_SMEM
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
GROUPS
cd "$GRAFT_REPO_ROOT" && python tools/pmc_parse.py "$OUT/sqc" > "$OUT/sqc_summary.txt" && cat "$OUT/sqc_summary.txt"
