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
// the output is in natural order.  All stages run in LDS (N complex64 = 8N bytes,
// N <= 2^14 -> <= 128 KiB of the 160 KiB); twiddles are an fp64-computed table
// rounded to fp32, read through the cache.  HBM traffic: the input segment once,
// the spectrum once.
#include "common.h"

namespace dsp {
namespace {

__device__ __forceinline__ unsigned bitrev(unsigned v, int log2n) {
  return log2n == 0 ? 0u : (__brev(v) >> (32 - log2n));
}

__device__ __forceinline__ void fft_stages(float2* __restrict__ buf, int log2n,
                                           const float2* __restrict__ tw) {
  const int half_n = (1 << log2n) >> 1;
  for (int s = 1; s <= log2n; ++s) {
    const int h = 1 << (s - 1);
    const int tshift = log2n - s;
    for (int i = threadIdx.x; i < half_n; i += blockDim.x) {
      const int k = i & (h - 1);
      const int j = ((i >> (s - 1)) << s) + k;
      const float2 w = tw[k << tshift];
      const float2 a = buf[j];
      const float2 o = buf[j + h];
      const float tr = fmaf(w.x, o.x, -w.y * o.y);
      const float ti = fmaf(w.x, o.y, w.y * o.x);
      buf[j] = make_float2(a.x + tr, a.y + ti);
      buf[j + h] = make_float2(a.x - tr, a.y - ti);
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
  const int64_t b = blockIdx.x;
  const float* xr = x + b * ld_x + seg_start;
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    const float v = (n < seg_len) ? xr[n] * win[n] : 0.f;
    buf[bitrev((unsigned)n, log2n)] = make_float2(v, 0.f);
  }
  __syncthreads();
  fft_stages(buf, log2n, tw);
  float* mr = mag + b * ld_mag;
  for (int k = threadIdx.x; k <= (N >> 1); k += blockDim.x) {
    const float2 v = buf[k];
    mr[k] = sqrtf(fmaf(v.x, v.x, v.y * v.y));
  }
}

__global__ __launch_bounds__(1024) void k_fft_c2c(
    const float* __restrict__ in, float* __restrict__ out, int log2n,
    int real_in, int64_t ld_in, int64_t ld_out, const float2* __restrict__ tw) {
  extern __shared__ __attribute__((aligned(16))) float2 buf[];
  const int N = 1 << log2n;
  const int64_t b = blockIdx.x;
  if (real_in) {
    const float* xr = in + b * ld_in;
    for (int n = threadIdx.x; n < N; n += blockDim.x)
      buf[bitrev((unsigned)n, log2n)] = make_float2(xr[n], 0.f);
  } else {
    const float2* xr = reinterpret_cast<const float2*>(in) + b * ld_in;
    for (int n = threadIdx.x; n < N; n += blockDim.x)
      buf[bitrev((unsigned)n, log2n)] = xr[n];
  }
  __syncthreads();
  fft_stages(buf, log2n, tw);
  float2* yr = reinterpret_cast<float2*>(out) + b * ld_out;
  for (int n = threadIdx.x; n < N; n += blockDim.x) yr[n] = buf[n];
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
  const size_t shm = (size_t)N * sizeof(float2);
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
  const size_t shm = (size_t)N * sizeof(float2);
  if (int rc = allow_lds(k_fft_c2c, shm)) return rc;
  TraceScope trace("fft", s);
  hipLaunchKernelGGL(k_fft_c2c, dim3((unsigned)B), dim3(threads_for(log2n)), shm, s, in,
                     out, log2n, real_in, ld_in, ld_out,
                     reinterpret_cast<const float2*>(tw));
  DSP_LAUNCHED("k_fft_c2c");
  return DSP_OK;
}

}  // namespace dsp
