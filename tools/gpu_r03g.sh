set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_g; mkdir -p $OUT
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; exit $rc; }
echo "== bench --gpus 2 (both ranks on device 0)"
DSP_BENCH_DEVICE=0 timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 2 > $OUT/bench_gpus2.json 2> $OUT/bench_gpus2.err || { tail -20 $OUT/bench_gpus2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_gpus2.json')); print('n_gpus', d['n_gpus'], 'per_gpu', d['config']['channels_per_gpu'], 'total', d['config']['total_channels'], 'value', d['value'], 'ms', d['ms_per_step'])"
