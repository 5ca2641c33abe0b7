# Round 4: config-5 persistent kernel -- parity tests, then same-box A/B of
# chained (path 2) vs persistent (path 3) per library build.
#   bash tools/gpu_gcp_ab.sh OUT lib ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nonfinite.py -m gpu -x -v \
  -k "config5 or generic or persistent or c5 or single_pass" --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for pass in 1 2; do
  for lib in "$@"; do
    for p in 2 3; do
      DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "${lib%.so}_path${p}_p$pass" \
        --config c5 --channels 8192 --steps 20 --path $p 2>&1 | grep -v amdgpu.ids >> $OUT/ab.log || exit 1
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
