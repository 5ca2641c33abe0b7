set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 python tools/iir_variants.py > gpurun_out/iir_variants.txt 2>&1 || { tail -20 gpurun_out/iir_variants.txt; exit 1; }
cat gpurun_out/iir_variants.txt
