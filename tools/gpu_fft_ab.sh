# Large-FFT A/B: tools/time_fft_nested.py over the main build and every
# lib/libdspcore_<variant>.so named on the command line, then the FFT parity tests.
#   bash tools/gpu_fft_ab.sh OUTDIR variant...
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
L=$PWD/dsp-audio-project_amd/lib
timeout -k 10 200 python -u tools/time_fft_nested.py 5 ${NEST:-23} ${SIZES:-24 25 26 27 28 29 30} > "$OUT/t_main.txt" 2>&1 || exit 1
for v in "$@"; do
  DSPCORE_LIB=$L/libdspcore_$v.so timeout -k 10 200 python -u tools/time_fft_nested.py 5 ${NEST:-23} ${SIZES:-24 25 26 27 28 29 30} > "$OUT/t_$v.txt" 2>&1 || exit 1
done
for f in "$OUT"/t_*.txt; do echo "== $f"; grep '^2' "$f"; done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nonfinite.py -x -q --timeout 240 --timeout-method thread -k "fft or spectrum or nonfinite" > "$OUT/pytest.log" 2>&1; rc=$?
tail -2 "$OUT/pytest.log"; exit $rc
