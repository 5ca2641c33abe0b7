# Round 5: config-5 persistent-kernel variants -- the config-5 / persistent
# parity tests on each variant library (DSPCORE_LIB), then same-box A/B
# (tools/gpu_ab_c5.sh: 8192 channels, dsp_chain_path(3)).
#   bash tools/gpu_gcp_var.sh OUT lib ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; rm -rf $OUT; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in "$@"; do
  DSPCORE_LIB="$L/$lib" timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nonfinite.py \
    tests/test_gpu_chain_contract.py -m gpu -x -q -k "config5 or generic or persistent or c5 or single_pass or extreme" \
    --timeout 300 --timeout-method thread > $OUT/pytest_${lib%.so}.log 2>&1 || { tail -30 $OUT/pytest_${lib%.so}.log; exit 1; }
  echo "$lib: $(tail -1 $OUT/pytest_${lib%.so}.log)"
done
bash tools/gpu_ab_c5.sh ${1%.so}_ab_tmp "$@" > /dev/null || exit 1
mv gpurun_out/${1%.so}_ab_tmp/ab.log $OUT/ab.log && rm -rf gpurun_out/${1%.so}_ab_tmp
python3 - $OUT/ab.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    try:
        d = json.loads(l)
    except ValueError:
        continue
    print(d["tag"], d["B"], d["handoff_ok"], d["step_ms"], d["kernels_ms"])
PY
