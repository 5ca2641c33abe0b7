# Config-5 phase ablations (tools/chain_ablation.py builds; results wrong by
# construction, timing only), same box, two alternations: chain_tile ms at 8192 ch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
for rep in 1 2; do
  for v in BASE NOSRC5 NOP1 NOSCAN NOP2 NOYST; do
    DSPCORE_LIB=$L/libdspcore_$v.so timeout -k 10 200 python tools/tile_ab.py --tag "c5_${v}_$rep" --config c5 --channels 8192 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
