# Multi-rank rehearsal of bench.py on a one-GPU box (every rank on cuda:0):
#   bash tools/gpu_mr.sh N [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
N=${1:-2}; shift
DSP_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus "$N" "$@"
