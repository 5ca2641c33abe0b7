set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab21
L=$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib
for rep in 1 2; do for v in "" _ts32 _nh8; do
  DSPCORE_LIB=$L/libdspcore$v.so timeout -k 10 120 python tools/ratio_sweep.py 4096 2/1 2/1:127 4/2 > gpurun_out/ab21/r${rep}$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab21/r${rep}$v.json'));print('$rep', '$v', [(r['L'],r['M'],r['K'],r['tile_len'],r['ms']) for r in d['rows']])"
done; done
