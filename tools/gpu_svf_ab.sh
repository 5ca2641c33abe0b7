# Same-box A/B of the float32 TPT-SVF stage 0 (-DDSP_SVF0=1 build) against the
# shipped chain kernel: config 4 (32768 ch) and config 3 (4096 ch), three
# alternations, then the +-15 dB precision tests on the variant.
# The variant was removed from csrc/ after this A/B (+4.8 %);
# the script stays as the record of how it was measured and no longer builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
L="$GRAFT_REPO_ROOT/dsp-audio-project_amd/lib"
mkdir -p gpurun_out/svf
for rep in 1 2 3; do
  for v in "" _svf0; do
    DSPCORE_LIB=$L/libdspcore$v.so timeout -k 10 300 python tools/tile_ab.py --tag "base${v}_$rep" --channels 32768 4096 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
python tools/tile_ab.py --compare base_1 base_svf0_1 || exit 1
DSPCORE_LIB=$L/libdspcore_svf0.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chain_contract.py -q -k "extreme_gains" --timeout 120 --timeout-method thread 2>&1 | tail -15
