# Round 4: the whole GPU suite, then a same-box A/B against a reference build.
#   bash tools/gpu_r04d.sh OUT ref.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$1; REF=$2; rm -rf gpurun_out/$OUT; mkdir -p gpurun_out/$OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$OUT/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest_gpu.log
bash tools/gpu_ab_only.sh $OUT $REF:0 libdspcore.so:0
