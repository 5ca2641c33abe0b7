// extern "C" entry points of libdspcore.so (declared in include/dspcore.h).
// Each one validates its arguments, launches on the caller's stream and
// returns a status code; nothing throws across the ABI.
#include <cstring>
#include <string>
#include <vector>

#include "common.h"

namespace dsp {

namespace {
thread_local std::string g_error;

struct TraceRec {
  const char* name;
  hipEvent_t start, stop;
};
struct TraceState {
  bool on = false;
  std::vector<TraceRec> recs;  // recs[0..used) are live
  size_t used = 0;
};
thread_local TraceState g_trace;
// dsp_chain_path: 0 single-pass kernel where instantiated (default), 1 always
// the two-launch chain, 2 / 3 the single-pass path with its chained-tile /
// persistent kernel (where one is built for the geometry), 4 the three-launch
// mode of the cascade alone (ABI 2.7).
thread_local int g_chain_path = 0;
// dsp_chain_spin_limit: polls before a single-pass hand-off wait gives up
// (2^23 polls with s_sleep 2 between them: ~0.4 s).
constexpr int64_t kDefaultSpins = (int64_t)1 << 23;
thread_local int64_t g_spin_limit = kDefaultSpins;
}  // namespace

TraceScope::TraceScope(const char* name, hipStream_t s) : slot_(-1), s_(s) {
  TraceState& t = g_trace;
  if (!t.on) return;
  if (t.used == t.recs.size()) {
    TraceRec r{name, nullptr, nullptr};
    if (hipEventCreate(&r.start) != hipSuccess || hipEventCreate(&r.stop) != hipSuccess) return;
    t.recs.push_back(r);
  }
  TraceRec& r = t.recs[t.used];
  r.name = name;
  if (hipEventRecord(r.start, s) != hipSuccess) return;
  slot_ = (int)t.used++;
}

TraceScope::~TraceScope() {
  if (slot_ >= 0) (void)hipEventRecord(g_trace.recs[slot_].stop, s_);
}

int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_error = buf;
  return code;
}

void clear_error() { g_error.clear(); }

}  // namespace dsp

extern "C" {

int dsp_version(void) {
  // 2.0.0: dsp_chain_f32 takes the tables' key and y may be NULL;
  // dsp_chain_tile_tables returns the key; the chain workspace holds the
  // single-pass region and the cascade's scratch side by side;
  // dsp_chain_status / dsp_chain_spin_limit added (round 3).
  // 2.1.0: every SRC entry point takes the caller's float32 taps and flushes
  // the sinc-zero noise itself (common.h, kTapFlushRel); inf and NaN input
  // propagate as through the reference's float64 convolution (round 4).
  // 2.2.0: dsp_pcm_batch_to_mono_f32 / dsp_pcm_batch_workspace_bytes (round 4).
  // 2.3.0: dsp_chain_path 2 / 3 pick the single-pass kernel variant (round 4).
  // 2.4.0: inf / NaN through the FFT and spectrum entry points get the
  // reference's labels (fft_nf.hip); dsp_fft_workspace_bytes adds the
  // four-step's per-row header; dsp_lfilter_nonfinite_f32 (round 5).
  // 2.5.0: DSP_MAX_LOG2N_FFT 28 -> 30 (nested four-step, round 5).
  // 2.6.0: dsp_lfilter_nonfinite_f32 scans x for a / a0 = [1, 0, ...];
  // single-pass chain kernels for every app ratio (round 6).
  // 2.7.0: dsp_chain_f32 takes the SRC bypass as the one-tap SRC (L = M = 1,
  // K = 1) single-pass, and mag == NULL skips the spectrum; dsp_chain_path 4;
  // dsp_chain_mode; dsp_convert_f64_f32 / dsp_convert_f32_f64; FFTs of 2^31
  // and 2^32 points (DSP_MAX_LOG2N_FFT 32, DSP_MAX_LOG2N_FOURSTEP 30) and the
  // dsp_fft_split_log2n test hook (round 6).
  return 20700;
}

const char* dsp_last_error(void) { return dsp::g_error.c_str(); }

int dsp_src_polyphase_f32(const float* x, float* y, int64_t B, int64_t n_in,
                          int64_t ld_x, int64_t n_out, int64_t ld_y,
                          const float* taps, int32_t K, int32_t L, int32_t M,
                          int64_t c_offset, void* stream) {
  dsp::clear_error();
  return dsp::launch_src(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, L, M, c_offset,
                         static_cast<hipStream_t>(stream));
}

size_t dsp_biquad_workspace_bytes(int64_t B, int64_t n, int32_t S,
                                  int64_t chunk_len) {
  return dsp::biquad_workspace_bytes(B, n, S, chunk_len);
}

int dsp_biquad_cascade_f32(const float* x, float* y, int64_t B, int64_t n,
                           int64_t ld_x, int64_t ld_y, const double* sos_host,
                           int32_t S, int32_t clip, int64_t chunk_len,
                           const double* state_table, void* workspace,
                           size_t workspace_bytes, void* stream) {
  dsp::clear_error();
  return dsp::launch_biquad(x, y, B, n, ld_x, ld_y, sos_host, S, clip, chunk_len,
                            state_table, workspace, workspace_bytes,
                            static_cast<hipStream_t>(stream));
}

int dsp_lfilter_nonfinite_f32(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x,
                              int64_t ld_y, const double* b, int32_t nb, const double* a,
                              int32_t na, void* stream) {
  dsp::clear_error();
  if (x && x == y) return dsp::set_error(DSP_EINVAL, "x and y must not alias");
  return dsp::launch_lfilter_nf(x, y, B, n, ld_x, ld_y, b, nb, a, na,
                                static_cast<hipStream_t>(stream));
}

size_t dsp_fft_workspace_bytes(int64_t B, int32_t log2n) {
  return dsp::fft_workspace_bytes(B, log2n);
}

int dsp_fft_split_log2n(int32_t log2n) {
  dsp::clear_error();
  if (log2n < -1 || (log2n >= 0 && (log2n < DSP_MAX_LOG2N + 2 || log2n > DSP_MAX_LOG2N_FOURSTEP + 1)))
    return dsp::set_error(DSP_EINVAL, "split log2n %d not in [%d, %d]", log2n, DSP_MAX_LOG2N + 2,
                          DSP_MAX_LOG2N_FOURSTEP + 1);
  return dsp::fft_split_log2n(log2n);
}

int dsp_fft_c2c_f32(const float* in, float* out, int64_t B, int32_t log2n,
                       int32_t real_input, int64_t ld_in, int64_t ld_out,
                       const float* twiddles, void* workspace, size_t workspace_bytes,
                       void* stream) {
  dsp::clear_error();
  return dsp::launch_fft(in, out, B, log2n, real_input, ld_in, ld_out, twiddles, workspace,
                         workspace_bytes, static_cast<hipStream_t>(stream));
}

int dsp_dft_size(int64_t n) {
  dsp::clear_error();
  if (n < 1 || n > DSP_MAX_DFT) return dsp::set_error(DSP_EINVAL, "n=%lld outside [1, %d]",
                                                      (long long)n, DSP_MAX_DFT);
  return 1 << dsp::bluestein_log2m(n);
}

int dsp_dft_f32(const float* in, float* out, int64_t B, int64_t n, int32_t real_input,
                int64_t ld_in, int64_t ld_out, const float* chirp, const float* chirp_fft,
                const float* twiddles_m, void* stream) {
  dsp::clear_error();
  return dsp::launch_dft(in, out, B, n, real_input, ld_in, ld_out, chirp, chirp_fft, twiddles_m,
                         static_cast<hipStream_t>(stream));
}

int dsp_spectrum_f32(const float* x, float* mag, int64_t B, int64_t ld_x,
                     int64_t seg_start, int64_t seg_len, int32_t log2n,
                     int64_t ld_mag, const float* window,
                     const float* twiddles, void* workspace, size_t workspace_bytes,
                     void* stream) {
  dsp::clear_error();
  return dsp::launch_spectrum(x, mag, B, ld_x, seg_start, seg_len, log2n, ld_mag,
                              window, twiddles, workspace, workspace_bytes,
                              static_cast<hipStream_t>(stream));
}

int dsp_stft_mag_f32(const float* x, float* mag, int64_t B, int64_t ld_x, int64_t seg_start,
                     int64_t seg_len, int64_t hop, int64_t frames, int32_t log2n,
                     int64_t ld_mag, const float* window, const float* twiddles,
                     void* stream) {
  dsp::clear_error();
  return dsp::launch_stft(x, mag, B, ld_x, seg_start, seg_len, hop, frames, log2n, ld_mag,
                          window, twiddles, static_cast<hipStream_t>(stream));
}

int dsp_chain_path(int32_t path) {
  dsp::clear_error();
  if (path < -1 || path > 4) return dsp::set_error(DSP_EINVAL, "chain path %d not in [-1, 4]", path);
  const int prev = dsp::g_chain_path;
  if (path >= 0) dsp::g_chain_path = path;
  return prev;
}

int64_t dsp_chain_tile_len(int64_t n_in, int64_t n_out, int32_t K, int32_t L, int32_t M,
                           int64_t c_offset, int32_t S) {
  return dsp::chain_tile_sub(n_in, n_out, K, L, M, c_offset, S);
}

int32_t dsp_chain_mode(int64_t B, int64_t n_in, int64_t n_out, int32_t K, int32_t L, int32_t M,
                       int64_t c_offset, int32_t S) {
  return dsp::chain_mode(B, n_in, n_out, K, L, M, c_offset, S);
}

size_t dsp_chain_workspace_bytes(int64_t B, int64_t n_in, int64_t n_out, int32_t K, int32_t L,
                                 int32_t M, int64_t c_offset, int32_t S, int64_t chunk_len) {
  // [status header + single-pass hand-off region][two-launch cascade scratch]:
  // the two paths never share bytes, so switching paths (dsp_chain_path, or a
  // geometry the single-pass kernel declines) cannot leave stale hand-off flags.
  const size_t head = dsp::chain_tile_workspace_bytes(B, n_in, n_out, K, L, M, c_offset, S);
  return dsp::add_sat(head, dsp::biquad_workspace_bytes(B, n_out, S, chunk_len));
}

int dsp_chain_status(void* workspace, size_t workspace_bytes, int32_t reset, void* stream) {
  dsp::clear_error();
  DSP_REQUIRE(workspace && workspace_bytes >= 4, "null or empty workspace");
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t word = 0;
  DSP_HIP(hipMemcpyAsync(&word, workspace, sizeof(word), hipMemcpyDeviceToHost, s));
  if (reset) DSP_HIP(hipMemsetAsync(workspace, 0, workspace_bytes, s));
  DSP_HIP(hipStreamSynchronize(s));
  return word != 0 ? 1 : 0;
}

int64_t dsp_chain_spin_limit(int64_t spins) {
  dsp::clear_error();
  if (spins < -1 || spins > 0xffffffffll)
    return dsp::set_error(DSP_EINVAL, "spin limit %lld not in [-1, 2^32)", (long long)spins);
  const int64_t prev = dsp::g_spin_limit;
  if (spins >= 0) dsp::g_spin_limit = spins;
  return prev;
}

size_t dsp_chain_tile_tables_bytes(void) { return dsp::chain_tile_tables_bytes(); }

int dsp_chain_tile_tables(void* tables_host, size_t tables_bytes, int64_t n_in, int64_t n_out,
                          const float* taps_host, int32_t K, int32_t L, int32_t M,
                          int64_t c_offset, const double* sos_host, int32_t S, uint64_t* key) {
  dsp::clear_error();
  return dsp::chain_tile_tables(tables_host, tables_bytes, n_in, n_out, taps_host, K, L, M,
                                c_offset, sos_host, S, key);
}

int dsp_chain_xstate_geometry(int64_t chunk_len, int32_t K, int32_t L, int32_t M,
                              int64_t c_offset, int64_t* shift, int64_t* q0, int64_t* rows) {
  dsp::clear_error();
  if (!shift || !q0 || !rows) return dsp::set_error(DSP_EINVAL, "null output pointer");
  return dsp::xstate_geometry(chunk_len, K, L, M, c_offset, shift, q0, rows);
}

int dsp_chain_f32(const float* x, float* y, float* z, float* mag, int64_t B, int64_t n_in,
                  int64_t ld_x, int64_t n_out, int64_t ld_y, const float* taps, int32_t K,
                  int32_t L, int32_t M, int64_t c_offset, const double* sos_host, int32_t S,
                  int32_t clip, int64_t chunk_len, const double* state_table,
                  const double* xstate_table, int64_t xstate_rows, const void* tile_tables,
                  uint64_t tile_key, int64_t seg_start,
                  int64_t seg_len, int32_t log2n, int64_t ld_mag, const float* window,
                  const float* twiddles, void* workspace, size_t workspace_bytes,
                  void* stream) {
  dsp::clear_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (y && y == z) return dsp::set_error(DSP_EINVAL, "y and z must not alias");
  if (log2n < 0 || log2n > DSP_MAX_LOG2N)
    return dsp::set_error(DSP_EINVAL, "chain spectrum log2n=%d outside [0, %d]", log2n,
                          DSP_MAX_LOG2N);
  if (B == 0) return DSP_OK;
  const size_t head = dsp::chain_tile_workspace_bytes(B, n_in, n_out, K, L, M, c_offset, S);
  DSP_REQUIRE(workspace && workspace_bytes >= head,
              "chain workspace too small: %zu < %zu bytes (dsp_chain_workspace_bytes)",
              workspace_bytes, head);
  int rc = dsp::kNotFused;
  if (dsp::g_chain_path != 1)
    rc = dsp::launch_chain_tile(x, y, z, B, n_in, ld_x, n_out, ld_y, taps, K, L, M, c_offset,
                                sos_host, S, clip, tile_tables, tile_key,
                                (uint32_t)dsp::g_spin_limit, dsp::g_chain_path, workspace, head,
                                s);
  if (rc == dsp::kNotFused) {
    // Two-launch chain: SRC, then the cascade with x-domain chunk states where
    // the input rows are aligned and the chunking fits, else the y-domain
    // table (include/dspcore.h).  y carries the SRC output between the two.
    if (!y)
      return dsp::set_error(DSP_EINVAL, "y == NULL needs the single-pass kernel (dsp_chain_tile_len "
                                        "> 0, its tables and key, dsp_chain_path 0)");
    char* scratch = static_cast<char*>(workspace) + head;
    const size_t scratch_bytes = workspace_bytes - head;
    rc = dsp::launch_src(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, L, M, c_offset, s);
    if (rc) return rc;
    if (xstate_table && dsp::xstate_applicable(n_out, S, chunk_len, x, ld_x, L, M))
      rc = dsp::launch_biquad_xstate(y, z, B, n_out, ld_y, ld_y, sos_host, S, clip, chunk_len, x,
                                     n_in, ld_x, K, L, M, c_offset, xstate_table, xstate_rows, s);
    else
      rc = dsp::launch_biquad(y, z, B, n_out, ld_y, ld_y, sos_host, S, clip, chunk_len,
                              state_table, scratch_bytes ? scratch : nullptr, scratch_bytes, s);
  }
  if (rc) return rc;
  if (!mag) return DSP_OK;  // (ABI 2.7) no spectrum asked for
  // after the clip z holds no inf, and NaN alone gives every bin NaN as in the
  // reference: the non-finite repair runs only when the cascade does not clip
  return dsp::launch_spectrum(z, mag, B, ld_y, seg_start, seg_len, log2n, ld_mag, window,
                              twiddles, nullptr, 0, s, clip == 0);
}

int dsp_wav_parse(const uint8_t* file, size_t len, dsp_wav_info* info) {
  dsp::clear_error();
  return dsp::wav_parse(file, len, info);
}

int dsp_audio_parse(const uint8_t* file, size_t len, dsp_wav_info* info) {
  dsp::clear_error();
  return dsp::audio_parse(file, len, info);
}

int dsp_pcm_to_mono_f32(const void* pcm, int32_t format, int32_t bits, int32_t channels,
                        int64_t B, int64_t frames, int64_t ld_bytes, float* out,
                        int64_t ld_out, void* stream) {
  dsp::clear_error();
  return dsp::launch_pcm_mono(pcm, format, bits, channels, B, frames, ld_bytes, out, ld_out,
                              static_cast<hipStream_t>(stream));
}

int dsp_peak_normalize_f32(float* x, int64_t B, int64_t n, int64_t ld, double threshold,
                           uint32_t* peak_out, void* stream) {
  dsp::clear_error();
  return dsp::launch_peak_normalize(x, B, n, ld, threshold, peak_out,
                                    static_cast<hipStream_t>(stream));
}

size_t dsp_pcm_batch_workspace_bytes(int64_t B, int64_t width) {
  return dsp::pcm_batch_workspace_bytes(B, width);
}

int dsp_pcm_batch_to_mono_f32(const void* pcm, size_t pcm_bytes, const dsp_pcm_row* rows,
                              int64_t B, int64_t width, float* out, int64_t ld_out,
                              double threshold, uint32_t* peak_out, void* workspace,
                              size_t workspace_bytes, void* stream) {
  dsp::clear_error();
  return dsp::launch_pcm_batch(pcm, pcm_bytes, rows, B, width, out, ld_out, threshold, peak_out,
                               workspace, workspace_bytes, static_cast<hipStream_t>(stream));
}

int dsp_quantize_pcm16(const float* z, int16_t* out, int64_t B, int64_t n, int64_t ld_z,
                       int64_t ld_out, uint32_t* peak_out, int32_t precision, void* stream) {
  dsp::clear_error();
  return dsp::launch_quantize_pcm16(z, out, B, n, ld_z, ld_out, peak_out, precision,
                                    static_cast<hipStream_t>(stream));
}

int dsp_convert_f64_f32(const double* in, float* out, int64_t n, void* stream) {
  dsp::clear_error();
  return dsp::launch_convert_f64_f32(in, out, n, static_cast<hipStream_t>(stream));
}

int dsp_convert_f32_f64(const float* in, double* out, int64_t n, void* stream) {
  dsp::clear_error();
  return dsp::launch_convert_f32_f64(in, out, n, static_cast<hipStream_t>(stream));
}

int dsp_wav_header_pcm16(uint8_t* header44, int32_t sample_rate, int32_t channels,
                         int64_t frames) {
  dsp::clear_error();
  return dsp::wav_header_pcm16(header44, sample_rate, channels, frames);
}

int dsp_trace_enable(int32_t enable) {
  dsp::clear_error();
  dsp::g_trace.on = enable != 0;
  dsp::g_trace.used = 0;
  return DSP_OK;
}

int dsp_trace_read(char* names, float* ms, int32_t max) {
  dsp::clear_error();
  auto& t = dsp::g_trace;
  int n = 0;
  for (size_t i = 0; i < t.used && n < max; ++i, ++n) {
    const auto& r = t.recs[i];
    DSP_HIP(hipEventSynchronize(r.stop));
    float v = 0.f;
    DSP_HIP(hipEventElapsedTime(&v, r.start, r.stop));
    if (ms) ms[n] = v;
    if (names) {
      std::strncpy(names + (size_t)n * DSP_TRACE_NAME, r.name, DSP_TRACE_NAME - 1);
      names[(size_t)n * DSP_TRACE_NAME + DSP_TRACE_NAME - 1] = 0;
    }
  }
  t.used = 0;
  return n;
}

}  // extern "C"
