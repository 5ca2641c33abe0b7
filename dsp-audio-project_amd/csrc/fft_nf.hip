// Non-finite input through the power-of-two FFT and the magnitude spectrum:
// the reference's inf / NaN labels, restored after the fast transforms.
//
// The reference transforms in complex128 with numpy's arithmetic
// (/root/reference/modules/dsp_core.py:41-66): a recursive radix-2 DIT whose
// butterflies are X[k] = E[k] + t, X[k + m/2] = E[k] - t with t = W * O[k],
// W = exp(-2j pi k / m), and numpy's complex product (a + bi)(c + di) =
// (ac - bd) + (ad + bc)i with no special case for infinities -- so inf * 0 =
// NaN wherever an infinite component meets the exactly-zero imaginary part of
// W at k = 0, and the spectrum's |X| (:91) is hypot: +inf when either
// component is infinite, NaN when one is NaN and none infinite.  The radix-16
// Stockham kernels (fft.hip) compute the same finite numbers in another
// order, so their inf / NaN labels differ.  What is restored here:
//
//   * the class (finite / +inf / -inf / NaN) of every output component is the
//     reference's.  Classes follow an algebra in which every finite number
//     acts as 0: sums are finite + finite = finite, inf + finite = inf,
//     inf - inf = NaN, NaN + anything = NaN; products by W's components (never
//     zero but for Im W at k = 0; signs: Re W > 0 for k <= m/4, the float64
//     cos(pi/2) = 6.1e-17 included, Im W < 0 for k > 0) keep or flip an inf,
//     turn it into NaN when the component is 0, and keep NaN.  The algebra is
//     commutative, associative and distributive, so the class of X[k] is the
//     class-sum, over the non-finite input components, of each one's
//     contribution along its unique path through the recursion: at level m
//     (m = 2 .. N, input bit log2(N/m) of n), an odd index multiplies by W_m^j,
//     j = k mod m/2, and negates when k mod m >= m/2; an even one passes
//     through.  nf_path below is that walk, evaluated in float arithmetic on
//     the values 0 / +-inf / NaN (which is the algebra: 0 * inf = NaN,
//     inf - inf = NaN).  tests/test_oracle_golden.py checks the same walk,
//     restated in numpy, against the oracle's recursion on random inputs;
//   * a component whose class is finite takes the DFT of the input with its
//     non-finite components set to zero -- exactly what the reference's
//     complex128 sums give there, since an inf or NaN never reaches it;
//   * for the spectrum, any non-finite windowed sample reaches a component of
//     every bin (every path multiplies by a non-zero Re W), so every |X[k]|
//     is +inf or NaN and no finite value is needed.
//
// Detection costs the fast path nothing up to DSP_MAX_LOG2N: every output of
// the Stockham kernels is a chain of adds and products by non-zero constants
// of every input, so one non-finite input makes X[0] (|X[0]|) non-finite, and
// k_nf_small reads X[0] of every transform, exits at once when all are finite
// and otherwise rebuilds the flagged transforms in LDS.  Above it the
// four-step's first step sets each row's flag in the header behind its
// workspace (and, for the complex transforms, reads non-finite components as
// zero, so its output already holds the finite values); k_nf_list gathers the
// flagged rows' non-finite inputs into the freed workspace and k_nf_fix
// rewrites the outputs from them.
#include "common.h"

namespace dsp {
namespace {

constexpr int kNfThreads = 256;

// Class code (common.h nf_code: 0 finite, 1 +inf, 2 -inf, 3 NaN) as the
// algebra's value.
__device__ __forceinline__ float nf_cls(int code) { return code == 0 ? 0.f : nf_value(code); }

// Input n of transform t, as the fast kernels read it: the spectrum's
// windowed segment sample (zero past the valid range), a real sample, or a
// complex value.
__device__ __forceinline__ float2 nf_input(const NfArgs& a, int64_t t, int64_t n) {
  if (a.mode == 2) {
    const int64_t row = a.frames == 1 ? t : t / a.frames;
    const int64_t f0 = (t - row * a.frames) * a.hop;
    const float s = (n < a.seg_len - f0) ? a.in[row * a.ld_in + a.seg_start + f0 + n] : 0.f;
    return make_float2(s * a.win[n], 0.f);
  }
  if (a.mode == 1) return make_float2(a.in[t * a.ld_in + n], 0.f);
  return reinterpret_cast<const float2*>(a.in)[t * a.ld_in + n];
}

// Packed list entry of input n with component classes (cr, ci), or 0 when
// both are finite: index << 4 | cr << 2 | ci (32-bit entries in k_nf_small's
// LDS, n < 2^14; 64-bit in the four-step's workspace lists, n < 2^30).
template <typename E>
__device__ __forceinline__ E nf_entry(int64_t n, float2 v) {
  const int cr = nf_code(v.x), ci = nf_code(v.y);
  return (cr | ci) ? ((E)n << 4) | (E)(cr << 2) | (E)ci : E(0);
}

// The class pair that input entry e contributes to X[k] (see the header).
__device__ __forceinline__ float2 nf_path(uint64_t e, uint32_t k, int lg) {
  const uint32_t n = (uint32_t)(e >> 4);
  float cr = nf_cls((e >> 2) & 3), ci = nf_cls(e & 3);
#pragma unroll 1
  for (int l = 1; l <= lg; ++l) {
    if (!((n >> (lg - l)) & 1)) continue;  // even: E passes through unchanged
    const uint32_t m = 1u << l, h = m >> 1;
    const uint32_t km = k & (m - 1), j = km & (h - 1);
    const float wr = j <= (m >> 2) ? 1.f : -1.f;
    const float wi = j == 0 ? 0.f : -1.f;
    float tr = wr * cr - wi * ci;
    float ti = wr * ci + wi * cr;
    if (km >= h) {
      tr = -tr;
      ti = -ti;
    }
    cr = tr;
    ci = ti;
  }
  return make_float2(cr, ci);
}

// Class-sum over the list for output k (stops once both components are NaN).
template <typename E>
__device__ __forceinline__ float2 nf_classes(const E* list, uint32_t count, uint32_t k, int lg) {
  float2 acc = make_float2(0.f, 0.f);
#pragma unroll 1
  for (uint32_t i = 0; i < count; ++i) {
    const float2 c = nf_path(list[i], k, lg);
    acc.x += c.x;
    acc.y += c.y;
    if (acc.x != acc.x && acc.y != acc.y) break;
  }
  return acc;
}

// Writes output k from its classes: a component with a non-finite class
// takes it; for the spectrum, hypot's rule.  Finite classes keep `out`.
__device__ __forceinline__ void nf_store(const NfArgs& a, int64_t t, uint32_t k, float2 c) {
  if (a.mode == 2) {
    const bool inf = __builtin_isinf(c.x) || __builtin_isinf(c.y);
    const bool nan = c.x != c.x || c.y != c.y;
    if (inf || nan) a.out[t * a.ld_out + k] = inf ? __builtin_inff() : __builtin_nanf("");
  } else {
    float* o = a.out + 2 * (t * a.ld_out + k);
    if (!__builtin_isfinite(c.x)) o[0] = c.x;
    if (!__builtin_isfinite(c.y)) o[1] = c.y;
  }
}

__device__ __forceinline__ float2 nf_cmul(float2 a, float2 w) {
  return make_float2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}

// Up to DSP_MAX_LOG2N: each workgroup checks X[0] of kNfThreads transforms
// and rebuilds the flagged ones, one at a time, with all its threads:
//   complex modes: the radix-2 DIT of the input with non-finite components
//     zeroed, in LDS (8 N bytes), written whole;
//   then the list of non-finite inputs (LDS, <= N entries) and, for every
//     output, the class-sum over it.
__global__ __launch_bounds__(kNfThreads) void k_nf_small(NfArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t nf_lds[];
  uint32_t* flagged = nf_lds;               // [kNfThreads]
  uint32_t* counts = nf_lds + kNfThreads;   // [0] flagged, [1] list entries
  float2* buf = reinterpret_cast<float2*>(nf_lds + kNfThreads + 4);
  uint32_t* list = nf_lds + kNfThreads + 4;
  const int tid = threadIdx.x;
  const int lg = a.log2n;
  const uint32_t N = 1u << lg;
  const uint32_t nout = a.mode == 2 ? N / 2 + 1 : N;
  if (tid == 0) counts[0] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kNfThreads;
  {
    const int64_t t = t0 + tid;
    if (t < a.B) {
      bool bad;
      if (a.mode == 2) {
        bad = !__builtin_isfinite(a.out[t * a.ld_out]);
      } else {
        const float2 v = reinterpret_cast<const float2*>(a.out)[t * a.ld_out];
        bad = !__builtin_isfinite(v.x) || !__builtin_isfinite(v.y);
      }
      if (bad) flagged[atomicAdd(&counts[0], 1u)] = (uint32_t)tid;
    }
  }
  __syncthreads();
  const uint32_t nflag = counts[0];
#pragma unroll 1
  for (uint32_t f = 0; f < nflag; ++f) {
    const int64_t t = t0 + flagged[f];
    __syncthreads();  // the previous transform's LDS reads are done
    if (a.mode != 2) {
      const float2* tw = reinterpret_cast<const float2*>(a.tw);
      for (uint32_t n = tid; n < N; n += kNfThreads) {
        float2 v = nf_input(a, t, n);
        if (!__builtin_isfinite(v.x)) v.x = 0.f;
        if (!__builtin_isfinite(v.y)) v.y = 0.f;
        buf[lg ? (__builtin_bitreverse32(n) >> (32 - lg)) : 0] = v;
      }
      __syncthreads();
      for (int l = 1; l <= lg; ++l) {
        const uint32_t h = 1u << (l - 1), m = h << 1;
        for (uint32_t i = tid; i < N / 2; i += kNfThreads) {
          const uint32_t j = i & (h - 1), g = (i - j) * 2;
          const float2 w = tw[(size_t)j * (N / m)];
          const float2 e = buf[g + j], o = nf_cmul(buf[g + j + h], w);
          buf[g + j] = make_float2(e.x + o.x, e.y + o.y);
          buf[g + j + h] = make_float2(e.x - o.x, e.y - o.y);
        }
        __syncthreads();
      }
      float2* o = reinterpret_cast<float2*>(a.out) + t * a.ld_out;
      for (uint32_t k = tid; k < N; k += kNfThreads) o[k] = buf[k];
      // the class stores below overwrite some of these from other threads
      __threadfence();
      __syncthreads();
    }
    if (tid == 0) counts[1] = 0;
    __syncthreads();
    for (uint32_t n = tid; n < N; n += kNfThreads) {
      const uint32_t e = nf_entry<uint32_t>(n, nf_input(a, t, n));
      if (e) list[atomicAdd(&counts[1], 1u)] = e;
    }
    __syncthreads();
    const uint32_t cnt = counts[1];
    if (cnt)
      for (uint32_t k = tid; k < nout; k += kNfThreads) nf_store(a, t, k, nf_classes(list, cnt, k, lg));
  }
}

// Above DSP_MAX_LOG2N.  hdr[2 r] = row r's flag (set by the four-step's first
// step), hdr[2 r + 1] = its list length; the list of row r is
// lists[r * list_stride ...] (64-bit entries).
__global__ __launch_bounds__(kNfThreads) void k_nf_list(NfArgs a, uint32_t* hdr, uint64_t* lists,
                                                        int64_t list_stride) {
  const int64_t r = blockIdx.y;
  if (!hdr[2 * r]) return;
  const int64_t N = int64_t(1) << a.log2n;
  uint64_t* list = lists + r * list_stride;
  for (int64_t n = (int64_t)blockIdx.x * kNfThreads + threadIdx.x; n < N;
       n += (int64_t)gridDim.x * kNfThreads) {
    const uint64_t e = nf_entry<uint64_t>(n, nf_input(a, r, n));
    if (e) list[atomicAdd(&hdr[2 * r + 1], 1u)] = e;
  }
}

__global__ __launch_bounds__(kNfThreads) void k_nf_fix(NfArgs a, const uint32_t* hdr,
                                                       const uint64_t* lists, int64_t list_stride) {
  const int64_t r = blockIdx.y;
  const uint32_t cnt = hdr[2 * r + 1];
  if (!hdr[2 * r] || !cnt) return;
  const int64_t N = int64_t(1) << a.log2n;
  const int64_t nout = a.mode == 2 ? N / 2 + 1 : N;
  const uint64_t* list = lists + r * list_stride;
  for (int64_t k = (int64_t)blockIdx.x * kNfThreads + threadIdx.x; k < nout;
       k += (int64_t)gridDim.x * kNfThreads)
    nf_store(a, r, (uint32_t)k, nf_classes(list, cnt, (uint32_t)k, a.log2n));
}

}  // namespace

int launch_nf_small(const NfArgs& a, hipStream_t s) {
  DSP_REQUIRE(a.log2n >= 0 && a.log2n <= DSP_MAX_LOG2N, "non-finite repair: log2n=%d", a.log2n);
  if (a.B == 0) return DSP_OK;
  const size_t N = size_t(1) << a.log2n;
  const size_t body = a.mode == 2 ? N * sizeof(uint32_t) : N * 8;
  const size_t shm = (kNfThreads + 4) * sizeof(uint32_t) + body;
  if (int rc = allow_lds(k_nf_small, shm)) return rc;
  hipLaunchKernelGGL(k_nf_small, dim3((unsigned)ceil_div(a.B, kNfThreads)), dim3(kNfThreads), shm,
                     s, a);
  DSP_LAUNCHED("k_nf_small");
  return DSP_OK;
}

int launch_nf_large(const NfArgs& a, uint32_t* hdr, uint64_t* lists, int64_t list_stride,
                    hipStream_t s) {
  DSP_REQUIRE(a.log2n > DSP_MAX_LOG2N && a.log2n <= DSP_MAX_LOG2N_FOURSTEP,
              "non-finite repair: log2n=%d", a.log2n);
  if (a.B == 0) return DSP_OK;
  DSP_REQUIRE(a.B <= 65535, "non-finite repair: %lld rows per launch", (long long)a.B);
  const int64_t N = int64_t(1) << a.log2n;
  // a bounded grid: the common case (no flagged row) exits at once per group
  const int64_t per_row = 2048 / a.B > 0 ? 2048 / a.B : 1;
  const unsigned gl = (unsigned)std::min<int64_t>(ceil_div(N, kNfThreads), per_row);
  hipLaunchKernelGGL(k_nf_list, dim3(gl, (unsigned)a.B), dim3(kNfThreads), 0, s, a, hdr, lists,
                     list_stride);
  DSP_LAUNCHED("k_nf_list");
  hipLaunchKernelGGL(k_nf_fix, dim3(gl, (unsigned)a.B), dim3(kNfThreads), 0, s, a,
                     static_cast<const uint32_t*>(hdr), static_cast<const uint64_t*>(lists),
                     list_stride);
  DSP_LAUNCHED("k_nf_fix");
  return DSP_OK;
}

}  // namespace dsp
