# Board power and clock under a pure HBM stream (tools/ubench_rw_mix --burn: the 1 read :
# 2 writes kernel back to back for 30 s) for comparison with the chain kernels (gpu_power.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/power_stream; rm -rf $OUT; mkdir -p $OUT
timeout -k 5 90 ./tools/ubench_rw_mix --burn 30 > $OUT/burn.txt 2>&1 &
pid=$!
i=0
while kill -0 $pid 2>/dev/null && [ $i -lt 30 ]; do
  sleep 2; i=$((i+1))
  { date +%s; rocm-smi --showpower --showclocks 2>&1; } > $OUT/load_$(printf %03d $i).txt || true
done
wait $pid || exit 1
for f in $OUT/load_*; do grep -iE "Power \(W\)|sclk" $f | sed 's/GPU\[0\]\t*: //' | tr '\n' ' '; echo; done
tail -3 $OUT/burn.txt
