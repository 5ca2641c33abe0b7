// Shared helpers for the libdspcore HIP sources (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cmath>
#include <cstdint>
#include <cstdio>

#include "dspcore.h"

namespace dsp {

// Thread-local error string behind dsp_last_error(): every entry point is
// reentrant and threads driving different GPUs never see each other's errors.
int set_error(int code, const char* fmt, ...);
void clear_error();

#define DSP_REQUIRE(cond, ...)                              \
  do {                                                      \
    if (!(cond)) return ::dsp::set_error(DSP_EINVAL, __VA_ARGS__); \
  } while (0)

#define DSP_HIP(expr)                                                        \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess)                                                    \
      return ::dsp::set_error(DSP_EHIP, "%s failed: %s", #expr,              \
                              hipGetErrorString(e_));                        \
  } while (0)

// Checks the launch that was just enqueued.
#define DSP_LAUNCHED(name)                                                   \
  do {                                                                       \
    hipError_t e_ = hipGetLastError();                                       \
    if (e_ != hipSuccess)                                                    \
      return ::dsp::set_error(DSP_EHIP, "launch of %s failed: %s", name,     \
                              hipGetErrorString(e_));                        \
  } while (0)

constexpr int kWave = 64;
constexpr int kNotFused = 1;  // a fast path's launcher declined; nothing was launched

// RAII bracket of one kernel launch for dsp_trace_* (no-op unless enabled on
// this thread).
class TraceScope {
 public:
  TraceScope(const char* name, hipStream_t s);
  ~TraceScope();
  TraceScope(const TraceScope&) = delete;
  TraceScope& operator=(const TraceScope&) = delete;

 private:
  int slot_;
  hipStream_t s_;
};

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// a * b * c * d in size_t, saturating at SIZE_MAX (a workspace nobody can
// allocate: the launch then fails its size check instead of wrapping).
inline size_t mul_sat(size_t a, size_t b, size_t c = 1, size_t d = 1) {
  size_t r;
  if (__builtin_mul_overflow(a, b, &r) || __builtin_mul_overflow(r, c, &r) ||
      __builtin_mul_overflow(r, d, &r))
    return SIZE_MAX;
  return r;
}
inline size_t add_sat(size_t a, size_t b) { return a > SIZE_MAX - b ? SIZE_MAX : a + b; }

// Dynamic LDS above 64 KiB must be opted into per kernel (gfx950 has 160 KiB).
template <typename Kern>
inline int allow_lds(Kern kernel, size_t bytes) {
  if (bytes > 65536)
    DSP_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)bytes));
  return DSP_OK;
}

// Resident workgroups on the device for a kernel (asked once per calling thread,
// kernel instance and launch shape; thread_local: no state shared between
// threads).  The kernel is a template argument so that every kernel has its
// own cache (as a function argument, every instance of one signature shared
// it); the cache is keyed by device, block size and LDS bytes (a kernel whose
// LDS depends on the call's geometry asks again when it changes).
template <auto K>
int resident_groups(int threads, size_t shm) {
  thread_local int dev = -1, cached = 0, cthreads = 0;
  thread_local size_t cshm = 0;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return 0;
  if (d != dev || cached <= 0 || threads != cthreads || shm != cshm) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(K),
                                                     threads, shm) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
      return 0;
    dev = d;
    cthreads = threads;
    cshm = shm;
    cached = per_cu * cus;
  }
  return cached;
}

// Workgroup barrier that waits only for LDS traffic.  __syncthreads() also
// drains outstanding global loads/stores (vmcnt(0)) on gfx950, which would
// serialise prefetches and stores with the barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Taps (include/dspcore.h, dsp_src_polyphase_f32).  The kernels' finite
// arithmetic uses the caller's float32 taps with every |t| <= kTapFlushRel *
// max|t| flushed to zero when L > 1: those are the float64 rounding noise of
// the reference's sinc at its zeros (dsp_core.py:120-129, sinc(k L / L) with
// |L h| ~ 1e-17 .. 1e-34, and the Blackman window's end taps), below 1e-14 of
// the signal in y, and flushing them makes the branch that holds the centre
// tap a pure delay (chain_tile.hip, DLY).  The caller's unflushed taps serve
// windows that hold an inf or NaN (nonfinite_sum below), so non-finite input
// propagates as through the reference's float64 convolution.
constexpr float kTapFlushRel = 1e-12f;

// Largest |t| that is flushed (negative: none, for L == 1).
inline float tap_flush_threshold(const float* taps, int K, int L) {
  if (L <= 1) return -1.f;
  float m = 0.f;
  for (int k = 0; k < K; ++k) m = fmaxf(m, fabsf(taps[k]));
  return kTapFlushRel * m;
}

__host__ __device__ __forceinline__ float flush_tap(float t, float thr) {
  return fabsf(t) <= thr ? 0.f : t;
}

// Non-finite inputs.  A window of the reference's convolution that holds an
// inf or NaN sums to the sum of its non-finite terms alone (finite terms
// cannot change an inf or a NaN; every reference tap is non-zero): +-inf when
// the infs that meet a tap agree in sign, NaN otherwise.  window_sums returns,
// for one output, nf = sum over t of taps[phi + L t] * xn(q - t) with xn = x's
// non-finite samples (finite ones zeroed) and the caller's unflushed taps --
// exactly the reference's result when the window holds an inf or NaN, +-0
// otherwise -- and fin = the kernels' canonical sum of the finite samples with
// the flushed taps: two FMA chains over x ascending, term t in chain
// (pb - t) & 1, fin = chain 0 + chain 1 (pb = q for the packed kernels, whose
// chains follow x's absolute parity; pb = T - 1 for the generic ones, whose
// chains follow the parity from the window start q - (T - 1)); pb < 0: one
// chain (the odd-M register-blocked kernel).  xat(t) returns x[q - t].
template <class XAT>
__device__ __forceinline__ void window_sums(const float* __restrict__ taps, int K, int L, int phi,
                                            float thr, int pb, XAT xat, float& nf, float& fin) {
  float sn = 0.f, c0 = 0.f, c1 = 0.f;
  // (the tap index in a VGPR even where it is wave-uniform: the rare path runs
  // inside kernels whose SGPRs are all taken)
  int t = (K - 1 - phi) / L;
  asm volatile("" : "+v"(t));
#pragma unroll 1
  for (; t >= 0; --t) {
    const float xv = xat(t), tv = taps[phi + L * t];
    const bool fx = __builtin_isfinite(xv);
    sn = fmaf(tv, fx ? 0.f : xv, sn);
    const float tf = flush_tap(tv, thr), xf = fx ? xv : 0.f;
    if (pb >= 0 && ((pb - t) & 1)) c1 = fmaf(tf, xf, c1);
    else c0 = fmaf(tf, xf, c0);
  }
  nf = sn;
  fin = pb >= 0 ? c0 + c1 : c0;
}

// The rare path's merge for one output: the reference's inf or NaN where the
// window holds one; else the kernel's sum y, unless that picked up a NaN
// through a zero tap that meets a neighbouring output's non-finite sample
// (packed tap pairs and class rows reach one or two samples past an output's
// window), in which case fin, the same canonical sum without that sample.
// Returns whether y is non-finite.
__device__ __forceinline__ bool nf_fix(float& y, float nf, float fin) {
  if (!__builtin_isfinite(nf)) {
    y = nf;
    return true;
  }
  if (!__builtin_isfinite(y)) y = fin;
  return false;
}

// Class code of a non-finite output (0: finite) and its value back.
__device__ __forceinline__ int nf_code(float v) {
  return __builtin_isfinite(v) ? 0 : (v != v ? 3 : (v > 0.f ? 1 : 2));
}
__device__ __forceinline__ float nf_value(int code) {
  return code == 1 ? __builtin_inff() : (code == 2 ? -__builtin_inff() : __builtin_nanf(""));
}

// fma(x, 0, acc) is NaN exactly when x is an inf or a NaN: accumulating it over
// the samples a thread loads flags non-finite input at one FMA per two values.
typedef float nf_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ nf_f32x2 nf_acc(nf_f32x2 acc, float4 v) {
  const nf_f32x2 z = {0.f, 0.f};
  acc = __builtin_elementwise_fma(nf_f32x2{v.x, v.y}, z, acc);
  return __builtin_elementwise_fma(nf_f32x2{v.z, v.w}, z, acc);
}
__device__ __forceinline__ bool nf_any(nf_f32x2 acc) { return !__builtin_isfinite(acc.x + acc.y); }

// A state that picked up an inf or NaN becomes all NaN: the reference's
// cascade (lfilter, DF2T) turns every later output into NaN after a non-finite
// input (b1 x - a1 y = inf - inf for the peaking sections, whose b1 == a1), and
// a carried state of +-infs could instead clip to +-1.
template <int D>
__device__ __forceinline__ void nf_poison(double (&e)[D]) {
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < D; ++i) s = fma(e[i], 0.0, s);
  if (!__builtin_isfinite(s)) {
#pragma unroll
    for (int i = 0; i < D; ++i) e[i] = __builtin_nan("");
  }
}

// Internal launchers shared by the entry points and the fused chain.
int launch_src(const float* x, float* y, int64_t B, int64_t n_in, int64_t ld_x,
               int64_t n_out, int64_t ld_y, const float* taps, int K, int L,
               int M, int64_t c, hipStream_t s);
int launch_biquad(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x,
                  int64_t ld_y, const double* sos, int S, int clip, int64_t chunk_len,
                  const double* state_table, void* ws, size_t ws_bytes, hipStream_t s);
int launch_spectrum(const float* x, float* mag, int64_t B, int64_t ld_x,
                    int64_t seg_start, int64_t seg_len, int log2n,
                    int64_t ld_mag, const float* window, const float* tw,
                    void* ws, size_t ws_bytes, hipStream_t s, bool repair = true);
// repair: run the non-finite repair (fft_nf.hip) after the transform; a caller
// whose input holds no inf (the chain after its clip: NaN alone already gives
// the reference's all-NaN spectrum) may skip it.  Above DSP_MAX_LOG2N the
// repair always runs.
int launch_stft(const float* x, float* mag, int64_t B, int64_t ld_x, int64_t seg_start,
                int64_t seg_len, int64_t hop, int64_t frames, int log2n, int64_t ld_mag,
                const float* window, const float* tw, hipStream_t s, bool repair = true);
int bluestein_log2m(int64_t n);
int launch_dft(const float* in, float* out, int64_t B, int64_t n, int real_in, int64_t ld_in,
               int64_t ld_out, const float* chirp, const float* chirp_fft, const float* tw_m,
               hipStream_t s);
int launch_fft(const float* in, float* out, int64_t B, int log2n, int real_in,
               int64_t ld_in, int64_t ld_out, const float* tw, void* ws, size_t ws_bytes,
               hipStream_t s);
size_t fft_workspace_bytes(int64_t B, int log2n);
size_t fourstep_workspace_bytes(int64_t B, int log2n);
// Above one four-step transform (fft_split.hip): the reference's top radix-2
// level (even / odd halves, then the butterfly); fft_split_log2n sets the
// calling thread's smallest log2n that takes it (a test hook; default
// DSP_MAX_LOG2N_FOURSTEP + 1) and returns the previous one.
bool fft_takes_split(int log2n);
int fft_split_log2n(int log2n);
size_t fft_split_workspace_bytes(int log2n);
int launch_fft_split(const float* in, float* out, int64_t B, int log2n, int real_in, int64_t ld_in,
                     int64_t ld_out, const float* tw, void* ws, size_t ws_bytes, hipStream_t s);

// Non-finite input through the power-of-two FFT / spectrum (fft_nf.hip): the
// reference's inf / NaN labels restored after the fast transform.  mode: 0
// complex rows in, 1 real rows in (both complex out), 2 windowed magnitude
// spectrum (segment / frame framing as dsp_stft_mag_f32).
struct NfArgs {
  const float* in;
  float* out;
  int64_t B, ld_in, ld_out;
  int64_t seg_start, seg_len, hop, frames;
  const float* win;
  const float* tw;
  int mode, log2n;
};
// log2n <= DSP_MAX_LOG2N: after any fast kernel (no workspace).
int launch_nf_small(const NfArgs& a, hipStream_t s);
// log2n > DSP_MAX_LOG2N, B <= 65535 rows: hdr (2 words per row: flag set by the
// four-step's first step, list length, both zeroed before it), lists (row r's
// at lists + r * list_stride 64-bit entries, >= N entries each).
int launch_nf_large(const NfArgs& a, uint32_t* hdr, uint64_t* lists, int64_t list_stride,
                    hipStream_t s);
size_t biquad_workspace_bytes(int64_t B, int64_t n, int S, int64_t chunk_len);
// lfilter's non-finite labels after the cascade (lfilter_nf.hip).
int launch_lfilter_nf(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x, int64_t ld_y,
                      const double* b, int nb, const double* a, int na, hipStream_t s);

// Audio I/O (audio_io.hip).
int wav_parse(const uint8_t* buf, size_t len, dsp_wav_info* info);
int aiff_parse(const uint8_t* buf, size_t len, dsp_wav_info* info);
int audio_parse(const uint8_t* buf, size_t len, dsp_wav_info* info);
int wav_header_pcm16(uint8_t* out, int32_t fs, int32_t channels, int64_t frames);
int launch_pcm_mono(const void* pcm, int format, int bits, int channels, int64_t B,
                    int64_t frames, int64_t ld_bytes, float* out, int64_t ld_out, hipStream_t s);
size_t pcm_batch_workspace_bytes(int64_t B, int64_t width);
int launch_pcm_batch(const void* pcm, size_t pcm_bytes, const dsp_pcm_row* rows, int64_t B,
                     int64_t width, float* out, int64_t ld_out, double threshold,
                     uint32_t* peak_out, void* ws, size_t ws_bytes, hipStream_t s);
int launch_peak_normalize(float* x, int64_t B, int64_t n, int64_t ld, double threshold,
                          uint32_t* peak, hipStream_t s);
int launch_convert_f64_f32(const double* in, float* out, int64_t n, hipStream_t s);
int launch_convert_f32_f64(const float* in, double* out, int64_t n, hipStream_t s);
int launch_quantize_pcm16(const float* z, int16_t* out, int64_t B, int64_t n, int64_t ld_z,
                          int64_t ld_out, uint32_t* peak, int precision, hipStream_t s);

// Chain fast path: pass 1 of the fused cascade reads the SRC input xs through
// the x-domain state table (include/dspcore.h, dsp_chain_xstate_geometry).
int xstate_geometry(int64_t chunk_len, int K, int L, int M, int64_t c, int64_t* shift,
                    int64_t* q0, int64_t* rows, int64_t* span = nullptr);
// Single-pass chain (chain_tile.hip): y = SRC(x) and z = clip(cascade(y)) in
// one launch, y never re-read.  chain_tile_sub returns the sub-chunk length of
// the instantiated geometry (0: the two-launch chain serves this call).
int64_t chain_tile_sub(int64_t n_in, int64_t n_out, int K, int L, int M, int64_t c, int S);
// The path dsp_chain_f32's default takes for a batch of B rows (0 two-launch,
// 1 single-pass, 3 the three-launch mode).
int chain_mode(int64_t B, int64_t n_in, int64_t n_out, int K, int L, int M, int64_t c, int S);
size_t chain_tile_workspace_bytes(int64_t B, int64_t n_in, int64_t n_out, int K, int L, int M,
                                  int64_t c, int S);
size_t chain_tile_tables_bytes();
int chain_tile_tables(void* out, size_t out_bytes, int64_t n_in, int64_t n_out, const float* taps,
                      int K, int L, int M, int64_t c, const double* sos, int S, uint64_t* key);
// y may be NULL (the y store is skipped).  variant: dsp_chain_path's setting
// (0 the launcher's choice, 2 chained tiles, 3 persistent).  Returns kNotFused (nothing
// launched) when the kernel does not serve the call or `key` is not the
// fingerprint of tables built for it.
int launch_chain_tile(const float* x, float* y, float* z, int64_t B, int64_t n_in, int64_t ld_x,
                      int64_t n_out, int64_t ld_y, const float* taps, int K, int L, int M,
                      int64_t c, const double* sos, int S, int clip, const void* tables,
                      uint64_t key, uint32_t max_spins, int variant, void* ws, size_t ws_bytes,
                      hipStream_t s);
// Whether launch_biquad_xstate's conditions on the cascade (n, S, chunk_len)
// and on the SRC input rows (16-byte aligned) hold.
bool xstate_applicable(int64_t n, int S, int64_t chunk_len, const float* xs, int64_t ld_xs,
                       int L, int M);
int launch_biquad_xstate(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x,
                         int64_t ld_y, const double* sos, int S, int clip, int64_t chunk_len,
                         const float* xs, int64_t n_in, int64_t ld_xs, int K, int L, int M,
                         int64_t c, const double* gx, int64_t gx_rows, hipStream_t s);

}  // namespace dsp
