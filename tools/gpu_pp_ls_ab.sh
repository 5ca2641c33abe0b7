# Ratio-sweep A/B of a per-phase geometry list variant (lib/libdspcore_<NAME>.so,
# tools/build_pp_variant.sh) against the shipped list: the ratios whose
# geometry differs, single-pass only, two alternations.
#   bash tools/gpu_pp_ls_ab.sh NAME RATIO...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
V=$1; shift
mkdir -p gpurun_out/ppab
for rep in 1 2; do
  for v in "" "_$V"; do
    DSPCORE_LIB=$L/libdspcore$v.so timeout -k 10 300 python tools/ratio_sweep.py 4096 "$@" > gpurun_out/ppab/r${rep}${v}.json 2> gpurun_out/ppab/err.txt || { tail -5 gpurun_out/ppab/err.txt; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ppab/r${rep}${v}.json'));print('$rep', '${v:-base}', ' '.join(f\"{r['L']}/{r['M']}:TS{r['tile_len']}:{r['ms']:.4f}\" for r in d['rows']))"
  done
done
