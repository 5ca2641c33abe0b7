# Board power and clocks while the chain runs back to back: read-only rocm-smi
# queries every 4 s beside a long bench run (config 4, then config 5), plus idle.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/power; mkdir -p $OUT
rocm-smi --showpower --showclocks --showmaxpower > $OUT/idle.txt 2>&1 || true
for c in c4 c5; do
  steps=6000; [ $c = c5 ] && steps=24000
  timeout -k 10 400 python bench.py --config $c --no-extras --cpu-per-proc 0 --steps $steps --warmup 5 > $OUT/bench_$c.json 2> $OUT/bench_$c.err &
  pid=$!
  i=0
  while kill -0 $pid 2>/dev/null && [ $i -lt 90 ]; do
    sleep 4; i=$((i+1))
    { date +%s; rocm-smi --showpower --showclocks 2>&1; } > $OUT/load_${c}_$(printf %03d $i).txt || true
  done
  wait $pid || { tail -5 $OUT/bench_$c.err; exit 1; }
done
echo "== idle"; grep -iE "power|sclk" $OUT/idle.txt | head -6
for c in c4 c5; do
  echo "== $c"; for f in $OUT/load_${c}_*; do grep -iE "Power \(W\)|sclk" $f | tr '\n' ' '; echo; done | sort | uniq -c | sort -rn | head -8
done
python -c "import json; [print(c, json.load(open('$OUT/bench_'+c+'.json'))['ms_per_step']) for c in ('c4','c5')]"
