# Round 4: persistent config-3/4 kernel (dsp_chain_path(3)) vs chained tiles (2):
# chain tests on path 3, then same-box A/B per build at 32768 / 16384 / 8192 / 4096 channels.
#   bash tools/gpu_tilep_ab.sh OUT lib ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; rm -rf $OUT; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for pass in 1 2; do
  for lib in "$@"; do
    for p in 2 3; do
      DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${lib%.so}_path${p}_p$pass" \
        --config c3 --channels 32768 8192 4096 --steps 20 --path $p 2>&1 | grep -v amdgpu.ids >> $OUT/ab.log || exit 1
    done
  done
done
python3 - $OUT/ab.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    try:
        d = json.loads(l)
    except ValueError:
        continue
    print(d["tag"], d["B"], d["handoff_ok"], d["step_ms"], d["kernels_ms"])
PY
python tools/tile_ab.py --compare libdspcore_path2_p1 libdspcore_path3_p1
python tools/tile_ab.py --compare libdspcore_path2_p1 libdspcore_tp1_path3_p1
