# Spectrum A/B: tools/tile_ab.py (chain + spectrum step, kernels from HIP events)
# at configs 3, 4 and 5 over the main build and lib/libdspcore_<variant>.so, two passes.
#   bash tools/gpu_spec_ab.sh OUTDIR variant...
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
L=$PWD/dsp-audio-project_amd/lib
for pass in 1 2; do for v in main "$@"; do for c in c3 c4 c5; do
  case $c in c3) ch=4096;; c4) ch=32768;; c5) ch=8192;; esac
  lib=""; [ "$v" = main ] || lib=$L/libdspcore_$v.so
  DSPCORE_LIB=$lib timeout -k 10 300 python tools/tile_ab.py --tag "${v}_${c}_p$pass" --config $c --channels $ch --steps 20 2>&1 | grep '^{' >> "$OUT/ab.log" || exit 1
done; done; done
python3 - "$OUT/ab.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["tag"], d["step_ms"], d["kernels_ms"])
PY
