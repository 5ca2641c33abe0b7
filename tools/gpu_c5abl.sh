# Config-5 phase ablations (tools/chain_ablation.py builds), same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/c5abl; mkdir -p $OUT
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for lib in libdspcore_BASE.so libdspcore_NOSCAN.so libdspcore_NOP1.so libdspcore_NOYST.so libdspcore_BASE.so; do
  DSPCORE_LIB="$L/$lib" timeout -k 10 300 python tools/tile_ab.py --tag "c5_${lib%.so}" --config c5 --channels 8192 2>&1 | grep -v amdgpu.ids | tee -a $OUT/c5abl.jsonl || exit 1
done
