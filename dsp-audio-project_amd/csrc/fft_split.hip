// FFTs above one four-step transform (2^31, 2^32 points): the reference's own
// top recursion level, on the device.
//
// fft_diezmado_en_tiempo (/root/reference/modules/dsp_core.py:41-66) splits x
// into its even and odd samples, transforms both halves and combines them:
//     t = W_N^k O[k],  X[k] = E[k] + t,  X[k + N/2] = E[k] - t,  k < N/2,
// with t the complex product (Re W Re O - Im W Im O) + (Re W Im O + Im W Re O) i
// (numpy's complex multiply).  Above DSP_MAX_LOG2N_FOURSTEP this file does
// exactly that level: k_split_gather writes the even and odd samples of the
// row contiguously into the workspace and the N/2-point twiddles (every
// second entry of the caller's N-point table: exp(-2 pi i 2k / N) is
// exp(-2 pi i k / (N/2)) bit for bit), launch_fft transforms the halves into
// the two halves of the output row (itself splitting again for 2^32), and
// k_split_combine runs the butterfly in place.  The halves' inf / NaN
// classes are the reference's (fft_nf.hip), and the combine's IEEE
// arithmetic on them is the reference's formula, so X's classes are too;
// finite values carry float32 rounding as everywhere (tests: 1e-5 max|X|).
// Rows one at a time; every index is 64-bit.
#include "common.h"

namespace dsp {
namespace {

thread_local int g_split_log2n = DSP_MAX_LOG2N_FOURSTEP + 1;

constexpr int kSplitNT = 256;
constexpr int64_t kSplitBlocks = 16384;

// even / odd samples of one row (real: floats; complex: float2), and the
// N/2-point twiddles tw_h[k] = tw[2k], k < N/4 (first grid-stride pass).
template <bool REAL>
__global__ __launch_bounds__(kSplitNT) void k_split_gather(const float* __restrict__ in,
                                                           float* __restrict__ even,
                                                           float* __restrict__ odd,
                                                           const float2* __restrict__ tw,
                                                           float2* __restrict__ tw_h, int64_t half) {
  const int64_t stride = (int64_t)gridDim.x * kSplitNT;
  for (int64_t i = (int64_t)blockIdx.x * kSplitNT + threadIdx.x; i < half; i += stride) {
    if constexpr (REAL) {
      const float2 p = reinterpret_cast<const float2*>(in)[i];  // x[2i], x[2i + 1]
      even[i] = p.x;
      odd[i] = p.y;
    } else {
      const float4 p = reinterpret_cast<const float4*>(in)[i];  // x[2i], x[2i + 1]
      reinterpret_cast<float2*>(even)[i] = make_float2(p.x, p.y);
      reinterpret_cast<float2*>(odd)[i] = make_float2(p.z, p.w);
    }
    if (i < half / 2) tw_h[i] = tw[2 * i];
  }
}

// X[k] = E[k] + W^k O[k], X[k + N/2] = E[k] - W^k O[k], in place over the row
// (E in its first half, O in its second).
__global__ __launch_bounds__(kSplitNT) void k_split_combine(float2* __restrict__ X,
                                                            const float2* __restrict__ tw,
                                                            int64_t half) {
  const int64_t stride = (int64_t)gridDim.x * kSplitNT;
  for (int64_t k = (int64_t)blockIdx.x * kSplitNT + threadIdx.x; k < half; k += stride) {
    const float2 e = X[k], o = X[k + half], w = tw[k];
    // numpy's complex product, not contracted into FMAs (the reference's
    // operation order for the inf / NaN classes)
    const float tr = __fsub_rn(__fmul_rn(w.x, o.x), __fmul_rn(w.y, o.y));
    const float ti = __fadd_rn(__fmul_rn(w.x, o.y), __fmul_rn(w.y, o.x));
    X[k] = make_float2(__fadd_rn(e.x, tr), __fadd_rn(e.y, ti));
    X[k + half] = make_float2(__fsub_rn(e.x, tr), __fsub_rn(e.y, ti));
  }
}

unsigned split_grid(int64_t n) {
  return (unsigned)std::min<int64_t>(ceil_div(n, (int64_t)kSplitNT), kSplitBlocks);
}

}  // namespace

int fft_split_log2n(int log2n) {
  const int prev = g_split_log2n;
  if (log2n >= 0) g_split_log2n = log2n;
  return prev;
}

bool fft_takes_split(int log2n) {
  return log2n > DSP_MAX_LOG2N_FOURSTEP ||
         (log2n >= g_split_log2n && log2n >= DSP_MAX_LOG2N + 2 && log2n <= DSP_MAX_LOG2N_FFT);
}

// [even: N/2 complex][odd: N/2 complex][tw_h: N/4 complex][the halves' own
// workspace], 256-byte aligned regions; rows reuse it.
size_t fft_split_workspace_bytes(int log2n) {
  const size_t half = (size_t)1 << (log2n - 1);
  const size_t a = (half * sizeof(float2) + 255) & ~(size_t)255;
  const size_t t = ((half / 2) * sizeof(float2) + 255) & ~(size_t)255;
  return add_sat(add_sat(2 * a, t), fft_workspace_bytes(1, log2n - 1) + 255);
}

int launch_fft_split(const float* in, float* out, int64_t B, int log2n, int real_in, int64_t ld_in,
                     int64_t ld_out, const float* tw, void* ws, size_t ws_bytes, hipStream_t s) {
  const size_t need = fft_split_workspace_bytes(log2n);
  DSP_REQUIRE(ws && ws_bytes >= need, "FFT workspace too small: %zu < %zu bytes", ws_bytes, need);
  DSP_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 255) == 0, "FFT workspace not 256-byte aligned");
  DSP_REQUIRE((reinterpret_cast<uintptr_t>(in) & (real_in ? 7 : 15)) == 0 && (ld_in % 2) == 0,
              "rows of a split FFT must start on 8 (real) / 16 (complex) bytes");
  const int64_t half = int64_t(1) << (log2n - 1);
  const size_t a = ((size_t)half * sizeof(float2) + 255) & ~(size_t)255;
  const size_t t = ((size_t)(half / 2) * sizeof(float2) + 255) & ~(size_t)255;
  char* base = static_cast<char*>(ws);
  float* even = reinterpret_cast<float*>(base);
  float* odd = reinterpret_cast<float*>(base + a);
  float2* tw_h = reinterpret_cast<float2*>(base + 2 * a);
  void* sub = base + 2 * a + t;
  const size_t sub_bytes = ws_bytes - (2 * a + t);
  for (int64_t b = 0; b < B; ++b) {
    const float* row = in + b * ld_in * (real_in ? 1 : 2);
    float2* X = reinterpret_cast<float2*>(out) + b * ld_out;
    {
      TraceScope trace("fft_split", s);
      if (real_in)
        hipLaunchKernelGGL(k_split_gather<true>, dim3(split_grid(half)), dim3(kSplitNT), 0, s, row,
                           even, odd, reinterpret_cast<const float2*>(tw), tw_h, half);
      else
        hipLaunchKernelGGL(k_split_gather<false>, dim3(split_grid(half)), dim3(kSplitNT), 0, s,
                           row, even, odd, reinterpret_cast<const float2*>(tw), tw_h, half);
      DSP_LAUNCHED("k_split_gather");
    }
    // the halves (the reference's pares / impares), into the row's halves
    if (int rc = launch_fft(even, reinterpret_cast<float*>(X), 1, log2n - 1, real_in, half, half,
                            reinterpret_cast<const float*>(tw_h), sub, sub_bytes, s))
      return rc;
    if (int rc = launch_fft(odd, reinterpret_cast<float*>(X + half), 1, log2n - 1, real_in, half,
                            half, reinterpret_cast<const float*>(tw_h), sub, sub_bytes, s))
      return rc;
    TraceScope trace("fft_split", s);
    hipLaunchKernelGGL(k_split_combine, dim3(split_grid(half)), dim3(kSplitNT), 0, s, X,
                       reinterpret_cast<const float2*>(tw), half);
    DSP_LAUNCHED("k_split_combine");
  }
  return DSP_OK;
}

}  // namespace dsp
