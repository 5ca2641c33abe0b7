# PMC passes (tools/pmc_chain.sh) of one workload for several library builds,
# same box -> gpurun_out/$TAG/<lib>/pmc_summary.txt.
#   bash tools/gpu_pmc_libs.sh TAG CONFIG "lib1.so lib2.so ..."
set -o pipefail
TAG=$1; CFG=$2; LIBS=$3
cd "$GRAFT_REPO_ROOT"
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in $LIBS; do
  DSPCORE_LIB="$L/$lib" bash tools/pmc_chain.sh "$TAG/${lib%.so}" 3 $CFG > /dev/null 2>&1 || { echo "pmc failed for $lib"; exit 1; }
  echo "== $lib"; grep -A24 "== spectrum" "gpurun_out/$TAG/${lib%.so}/pmc_summary.txt"
done
