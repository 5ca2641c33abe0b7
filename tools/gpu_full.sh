# Round measurement: GPU parity tests, smoke, full bench (with CPU baseline),
# rocprofv3 kernel stats of the bench, PMC passes -> gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-r01}
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
rm -rf "$OUT"; mkdir -p "$OUT"
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "== bench"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "== rocprof stats"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --cpu-per-proc 0 --no-config3 --config c3 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
cat "$OUT/kernel_stats.csv" | cut -d, -f1-8 | head -12
echo "== pmc"
mkdir -p "$OUT/pmc"
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group -d "$OUT/pmc/p$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/kernels_once.py" 3 > "$OUT/pmc/p$i.log" 2>&1 || { tail -20 "$OUT/pmc/p$i.log"; exit 1; }
done <<'GROUPS'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F64 SQ_INSTS_SALU SQ_INSTS_SMEM
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum
GROUPS
cd "$GRAFT_REPO_ROOT" && python tools/pmc_parse.py "$OUT/pmc" > "$OUT/pmc_summary.txt" && grep -E "^==|traffic" "$OUT/pmc_summary.txt"
