# PMC passes (one rocprofv3 --pmc run per counter group) over tools/kernels_once.py
# -> gpurun_out/$TAG/pmc, summarised by tools/pmc_parse.py.
#   bash tools/pmc_chain.sh TAG [kernels_once args...]
set -o pipefail
TAG=${1:-pmc}
shift
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT/pmc"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $group -d "$OUT/pmc/p$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/kernels_once.py" "$@" > "$OUT/pmc/p$i.log" 2>&1 || { tail -20 "$OUT/pmc/p$i.log"; exit 1; }
done <<'GROUPS'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F64 SQ_INSTS_SALU SQ_INSTS_SMEM
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_FMA_F32 GRBM_GUI_ACTIVE
GROUPS
cd "$GRAFT_REPO_ROOT" && python tools/pmc_parse.py "$OUT/pmc" > "$OUT/pmc_summary.txt" && cat "$OUT/pmc_summary.txt"
