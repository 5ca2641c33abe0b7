# Round 4: config-5 persistent kernels -- parity subset on each build, then the
# same-box A/B of path 2 (chained) vs path 3 (persistent) per build.
#   bash tools/gpu_gcq_ab.sh OUT lib ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; rm -rf $OUT; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in "$@"; do
  DSPCORE_LIB="$L/$lib" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nonfinite.py \
    tests/test_gpu_chain_contract.py -m gpu -x -q -k "config5 or generic or persistent or c5 or single_pass or handoff" \
    --timeout 300 --timeout-method thread > $OUT/pytest_${lib%.so}.log 2>&1 || { tail -30 $OUT/pytest_${lib%.so}.log; exit 1; }
  echo "$lib: $(tail -1 $OUT/pytest_${lib%.so}.log)"
done
for pass in 1 2; do
  for lib in "$@"; do
    for p in 2 3; do
      DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${lib%.so}_path${p}_p$pass" \
        --config c5 --channels 8192 2048 --steps 20 --path $p 2>&1 | grep -v amdgpu.ids >> $OUT/ab.log || exit 1
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
python tools/tile_ab.py --compare libdspcore_path2_p1 libdspcore_gcq_path3_p1
