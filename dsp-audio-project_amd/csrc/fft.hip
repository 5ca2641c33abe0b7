// Batched radix-2 decimation-in-time FFT and windowed magnitude spectrum for
// gfx950, one LDS-resident transform per workgroup.
//
// Replaces reference modules/dsp_core.py:41-66 (fft_diezmado_en_tiempo, a
// recursive radix-2 DIT in pure Python: 2N-1 calls, each building exp(-2j*pi*k/N)
// and concatenating E + W*O, E - W*O) and dsp_core.py:74-98
// (calcular_espectro_magnitud: centre segment or zero-padded input, Hann window,
// FFT, |X[k]| for k <= N/2).
//
// The recursion unrolls to the classic iterative form: load the input in
// bit-reversed order, then log2(N) butterfly stages of span 1, 2, 4, ... with
// twiddles W_N^(k*N/2^s); that is exactly the reference's concatenation order, so
// the output is in natural order.  All stages run in LDS: the data (N complex64,
// padded one slot per 32 rows so the bit-reversed scatter is conflict-free) and
// the N/2 twiddles (an fp64-computed table rounded to fp32, staged once per
// block for N <= 2^13; read through the cache for 2^14).  HBM traffic: the input
// segment once, the spectrum once.
#include "common.h"

namespace dsp {
namespace {

__device__ __forceinline__ unsigned bitrev(unsigned v, int log2n) {
  return log2n == 0 ? 0u : (__brev(v) >> (32 - log2n));
}

// LDS layout: element i lives at pad(i) = i + (i >> sh), sh = max(log2n - 5, 1).
// The bit-reversed scatter of 32 consecutive inputs then hits 32 different bank
// pairs (N >= 1024), and butterfly partners stay contiguous within a row.
__device__ __forceinline__ int pad_shift(int log2n) { return log2n > 6 ? log2n - 5 : 1; }
__device__ __forceinline__ int pad(int i, int sh) { return i + (i >> sh); }
constexpr int kTwLdsMaxLog2 = 13;  // larger transforms read twiddles through the cache
inline size_t lds_floats2(int log2n) {
  const int n = 1 << log2n;
  const int sh = log2n > 6 ? log2n - 5 : 1;
  const size_t tw = log2n <= kTwLdsMaxLog2 ? (size_t)(n > 1 ? n / 2 : 1) : 0;
  return (size_t)n + (size_t)(n >> sh) + tw;  // data + twiddles
}

// Copies the N/2 twiddles into LDS (float4 = two twiddles per load).
__device__ __forceinline__ void load_twiddles(float2* __restrict__ stw,
                                              const float2* __restrict__ tw, int log2n) {
  const int half_n = (1 << log2n) >> 1;
  if (half_n >= 2) {
    const float4* t4 = reinterpret_cast<const float4*>(tw);
    float4* s4 = reinterpret_cast<float4*>(stw);
    for (int i = threadIdx.x; i < half_n / 2; i += blockDim.x) s4[i] = t4[i];
  } else if (half_n == 1 && threadIdx.x == 0) {
    stw[0] = tw[0];
  }
}

__device__ __forceinline__ void fft_stages(float2* __restrict__ buf, int log2n, int sh,
                                           const float2* stw) {
  const int half_n = (1 << log2n) >> 1;
  for (int s = 1; s <= log2n; ++s) {
    const int h = 1 << (s - 1);
    const int tshift = log2n - s;
    for (int i = threadIdx.x; i < half_n; i += blockDim.x) {
      const int k = i & (h - 1);
      const int j = ((i >> (s - 1)) << s) + k;
      const float2 w = stw[k << tshift];
      const int pj = pad(j, sh), pk = pad(j + h, sh);
      const float2 a = buf[pj];
      const float2 o = buf[pk];
      const float tr = fmaf(w.x, o.x, -w.y * o.y);
      const float ti = fmaf(w.x, o.y, w.y * o.x);
      buf[pj] = make_float2(a.x + tr, a.y + ti);
      buf[pk] = make_float2(a.x - tr, a.y - ti);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(1024) void k_spectrum(
    const float* __restrict__ x, float* __restrict__ mag, int64_t ld_x,
    int64_t seg_start, int64_t seg_len, int log2n, int64_t ld_mag,
    const float* __restrict__ win, const float2* __restrict__ tw) {
  extern __shared__ __attribute__((aligned(16))) float2 buf[];
  const int N = 1 << log2n;
  const int sh = pad_shift(log2n);
  float2* stw = buf + (N + (N >> sh) + 1) / 2 * 2;  // 16-byte aligned
  const int64_t b = blockIdx.x;
  const float* xr = x + b * ld_x + seg_start;
  const bool tw_lds = log2n <= kTwLdsMaxLog2;
  if (tw_lds) load_twiddles(stw, tw, log2n);
  const float2* twp = tw_lds ? stw : tw;
  // Loads are issued 4 rows at a time with clamped (always valid) addresses
  // and masked afterwards, so they overlap instead of waiting one by one.
  if (seg_len > 0) {
    const int last = (int)seg_len - 1;
    for (int n0 = threadIdx.x; n0 < N; n0 += 4 * blockDim.x) {
      float a[4], w[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + r * blockDim.x;
        const int nc = n < N ? n : N - 1;
        a[r] = xr[nc < last ? nc : last];
        w[r] = win[nc];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + r * blockDim.x;
        if (n < N)
          buf[pad((int)bitrev((unsigned)n, log2n), sh)] =
              make_float2(n < seg_len ? a[r] * w[r] : 0.f, 0.f);
      }
    }
  } else {
    for (int n = threadIdx.x; n < N; n += blockDim.x) buf[pad(n, sh)] = make_float2(0.f, 0.f);
  }
  __syncthreads();
  fft_stages(buf, log2n, sh, twp);
  float* mr = mag + b * ld_mag;
  for (int k = threadIdx.x; k <= (N >> 1); k += blockDim.x) {
    const float2 v = buf[pad(k, sh)];
    mr[k] = sqrtf(fmaf(v.x, v.x, v.y * v.y));
  }
}

__global__ __launch_bounds__(1024) void k_fft_c2c(
    const float* __restrict__ in, float* __restrict__ out, int log2n,
    int real_in, int64_t ld_in, int64_t ld_out, const float2* __restrict__ tw) {
  extern __shared__ __attribute__((aligned(16))) float2 buf[];
  const int N = 1 << log2n;
  const int sh = pad_shift(log2n);
  float2* stw = buf + (N + (N >> sh) + 1) / 2 * 2;
  const int64_t b = blockIdx.x;
  const bool tw_lds = log2n <= kTwLdsMaxLog2;
  if (tw_lds) load_twiddles(stw, tw, log2n);
  const float2* twp = tw_lds ? stw : tw;
  for (int n0 = threadIdx.x; n0 < N; n0 += 4 * blockDim.x) {
    float2 a[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + r * blockDim.x;
      const int nc = n < N ? n : N - 1;
      if (real_in)
        a[r] = make_float2(in[b * ld_in + nc], 0.f);
      else
        a[r] = reinterpret_cast<const float2*>(in)[b * ld_in + nc];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + r * blockDim.x;
      if (n < N) buf[pad((int)bitrev((unsigned)n, log2n), sh)] = a[r];
    }
  }
  __syncthreads();
  fft_stages(buf, log2n, sh, twp);
  float2* yr = reinterpret_cast<float2*>(out) + b * ld_out;
  for (int n = threadIdx.x; n < N; n += blockDim.x) yr[n] = buf[pad(n, sh)];
}

int threads_for(int log2n) {
  const int half_n = (1 << log2n) >> 1;
  int nt = half_n < 64 ? 64 : half_n;
  if (nt > 256 && log2n <= 12) nt = 256;
  if (nt > 1024) nt = 1024;
  return nt;
}

}  // namespace

int launch_spectrum(const float* x, float* mag, int64_t B, int64_t ld_x,
                    int64_t seg_start, int64_t seg_len, int log2n,
                    int64_t ld_mag, const float* window, const float* tw,
                    hipStream_t s) {
  DSP_REQUIRE(log2n >= 0 && log2n <= DSP_MAX_LOG2N, "log2n=%d outside [0, %d]", log2n,
              DSP_MAX_LOG2N);
  const int64_t N = int64_t(1) << log2n;
  DSP_REQUIRE(B >= 0 && seg_start >= 0 && seg_len >= 0 && seg_len <= N,
              "bad segment start=%lld len=%lld (N=%lld)", (long long)seg_start,
              (long long)seg_len, (long long)N);
  DSP_REQUIRE(ld_mag >= N / 2 + 1, "ld_mag too small");
  DSP_REQUIRE(ld_x >= seg_start + seg_len, "segment exceeds the row");
  if (B == 0) return DSP_OK;
  DSP_REQUIRE(x && mag && window && tw, "null pointer");
  const size_t shm = (lds_floats2(log2n) + 2) * sizeof(float2);
  if (shm > 160 * 1024) return set_error(DSP_ENOTSUP, "FFT of 2^%d does not fit in LDS", log2n);
  if (int rc = allow_lds(k_spectrum, shm)) return rc;
  TraceScope trace("spectrum", s);
  hipLaunchKernelGGL(k_spectrum, dim3((unsigned)B), dim3(threads_for(log2n)), shm, s, x,
                     mag, ld_x, seg_start, seg_len, log2n, ld_mag, window,
                     reinterpret_cast<const float2*>(tw));
  DSP_LAUNCHED("k_spectrum");
  return DSP_OK;
}

int launch_fft(const float* in, float* out, int64_t B, int log2n, int real_in,
               int64_t ld_in, int64_t ld_out, const float* tw, hipStream_t s) {
  DSP_REQUIRE(log2n >= 0 && log2n <= DSP_MAX_LOG2N, "log2n=%d outside [0, %d]", log2n,
              DSP_MAX_LOG2N);
  const int64_t N = int64_t(1) << log2n;
  DSP_REQUIRE(B >= 0 && ld_in >= N && ld_out >= N, "bad sizes");
  if (B == 0) return DSP_OK;
  DSP_REQUIRE(in && out && tw, "null pointer");
  DSP_REQUIRE((reinterpret_cast<uintptr_t>(out) & 7) == 0 &&
                  (real_in || (reinterpret_cast<uintptr_t>(in) & 7) == 0),
              "complex buffers must be 8-byte aligned");
  const size_t shm = (lds_floats2(log2n) + 2) * sizeof(float2);
  if (shm > 160 * 1024) return set_error(DSP_ENOTSUP, "FFT of 2^%d does not fit in LDS", log2n);
  if (int rc = allow_lds(k_fft_c2c, shm)) return rc;
  TraceScope trace("fft", s);
  hipLaunchKernelGGL(k_fft_c2c, dim3((unsigned)B), dim3(threads_for(log2n)), shm, s, in,
                     out, log2n, real_in, ld_in, ld_out,
                     reinterpret_cast<const float2*>(tw));
  DSP_LAUNCHED("k_fft_c2c");
  return DSP_OK;
}

}  // namespace dsp
