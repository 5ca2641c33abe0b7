# Same-box A/B of a library variant (lib/libdspcore_<NAME>.so) against the
# shipped build on configs 4, 3 (tools/tile_ab.py --config c3: 32768 / 4096 ch)
# and 5 (8192 ch), three alternations, then the z comparison.
#   bash tools/gpu_var_ab.sh NAME
set -o pipefail
cd "$GRAFT_REPO_ROOT"
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
V=$1
for rep in 1 2 3; do
  for v in "" "_$V"; do
    DSPCORE_LIB=$L/libdspcore$v.so timeout -k 10 300 python tools/tile_ab.py --tag "ab${v}_$rep" --channels 32768 4096 2>&1 | grep -v amdgpu.ids || exit 1
    DSPCORE_LIB=$L/libdspcore$v.so timeout -k 10 300 python tools/tile_ab.py --tag "ab5${v}_$rep" --config c5 --channels 8192 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
python tools/tile_ab.py --compare ab_1 "ab_${V}_1" && python tools/tile_ab.py --compare ab5_1 "ab5_${V}_1"
