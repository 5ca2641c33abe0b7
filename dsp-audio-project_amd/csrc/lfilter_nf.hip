// Non-finite input through aplicar_ecuacion_diferencias' recursion: the
// labels scipy.signal.lfilter gives (/root/reference/modules/dsp_core.py:214).
//
// With len(a) > 1 lfilter runs the direct form II transposed recursion over
// b / a0 and a / a0, both zero-padded to D + 1 = max(len(a), len(b)):
//     y[k]   = z0 + b0 x[k]
//     z_i    = z_(i+1) + b_(i+1) x[k] - a_(i+1) y[k]      (i < D - 1)
//     z_(D-1) = b_D x[k] - a_D y[k]
// in float64.  From the first non-finite x[k0] on, every y is non-finite (y[k0]
// = b0 * inf or NaN; the state then holds a_i * y, and a non-finite value
// never becomes finite again through + and *), but whether a y is +inf, -inf
// or NaN depends on the coefficients' signs and zeros (0 * inf = NaN, a padded
// a_i or b_i included): a one-pole low-pass keeps +inf forever, the peaking
// sections (b1 == a1) turn it into NaN at once.  The cascade kernels (iir.hip)
// compute the filter as float64 second-order sections and make every output
// after a non-finite one NaN (common.h nf_poison), which is the reference's
// labelling for the EQ's peaking bands but not for every (b, a).
//
// k_lfilter_nf restores lfilter's labels after the cascade: one wave per row
// reads y[n-1] (the cascade leaves it non-finite exactly when x held an inf or
// NaN) and exits when it is finite -- except when a / a0 = [1, 0, ...], whose
// finite values the caller computed as a convolution (design.py 'fir_rec':
// y[n-1] is finite again len(b) samples after an inf), where every row scans
// x; a flagged row finds k0, then runs the
// recursion above on CLASSES -- finite values as 0, +-inf, NaN; coefficients
// as their signs +-1 or 0 -- which is lfilter's own inf / NaN arithmetic (the
// class of a sum or product does not depend on finite magnitudes), with the
// state in LDS and the lanes updating it in parallel, and writes y[k] for k >=
// k0.  Once every state is NaN, every later y is NaN and the wave fills the
// rest of the row.  The class state of a stretch of finite x evolves on its
// own; when a whole chunk of finite x leaves it where the chunk started, the
// labels repeat with the chunk (period | 64), and later chunks of finite x are
// filled from the previous one without running the recursion (a one-pole
// low-pass keeps +inf forever, a negative pole alternates its sign: without
// this, millions of samples ran one by one).
#include "common.h"

namespace dsp {
namespace {

constexpr int kLfWords = (DSP_LFILTER_NF_MAX + 1 + 15) / 16;

struct LfNfArgs {
  const float* x;
  float* y;
  int64_t B, n, ld_x, ld_y;
  int D;  // recursion order: max(len(a), len(b)) - 1, 1..DSP_LFILTER_NF_MAX
  int scan_x;  // a / a0 = [1, 0, ...]: y[n-1] says nothing, scan every row's x
  // signs of b / a0 and a / a0, 2 bits each (0: zero, 1: +, 2: -), 16 a word
  uint32_t b[kLfWords], a[kLfWords];
};

__device__ __forceinline__ float lf_sign(const uint32_t* w, int i) {
  const uint32_t c = (w[i >> 4] >> (2 * (i & 15))) & 3u;
  return c == 0 ? 0.f : (c == 1 ? 1.f : -1.f);
}

__device__ __forceinline__ float lf_cls(float v) {
  return __builtin_isfinite(v) ? 0.f : v;  // +-inf and NaN are their own class
}

__device__ __forceinline__ bool lf_same(float u, float v) {
  return u == v || (u != u && v != v);  // classes: 0, +-inf, NaN
}

// Orders this wave's LDS accesses (they execute in order within a wave; this
// keeps the compiler from moving them across the state update).
__device__ __forceinline__ void lf_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(kWave) void k_lfilter_nf(LfNfArgs p) {
  extern __shared__ float zs[];  // three state buffers of D: current, next, chunk start
  const int64_t r = blockIdx.x;
  const int lane = threadIdx.x;
  const int D = p.D;
  const float* x = p.x + r * p.ld_x;
  float* y = p.y + r * p.ld_y;
  if (!p.scan_x && __builtin_isfinite(y[p.n - 1])) return;
  // k0: the first non-finite input
  int64_t k0 = -1;
  for (int64_t base = 0; base < p.n && k0 < 0; base += kWave) {
    const int64_t k = base + lane;
    const bool bad = k < p.n && !__builtin_isfinite(x[k]);
    const uint64_t m = __ballot(bad);
    if (m) k0 = base + __builtin_ctzll(m);
  }
  if (k0 < 0) return;  // (a NaN the cascade made from finite input: nothing to relabel)
  for (int i = lane; i < 2 * D; i += kWave) zs[i] = 0.f;
  const float b0 = lf_sign(p.b, 0);
  float* cur = zs;
  float* nxt = zs + D;
  float* start = zs + 2 * D;
  int64_t c = k0 - (k0 % kWave);  // chunk of kWave samples: lane j holds x[c + j], y[c + j]
  bool saturated = false;
  bool periodic = false;  // the last chunk's labels repeat while x stays finite
  float yprev = 0.f;
#pragma unroll 1
  for (; c < p.n && !saturated; c += kWave) {
    const int64_t kl = c + lane;
    const float xv = kl < p.n ? x[kl] : 0.f;
    const bool fin = __ballot(!__builtin_isfinite(xv)) == 0;
    if (periodic && fin) {
      if (kl < p.n) y[kl] = yprev;  // (the state is unchanged)
      continue;
    }
    periodic = false;
    lf_order();
    for (int i = lane; i < D; i += kWave) start[i] = cur[i];
    float ymine = 0.f;
    const int j0 = c < k0 ? (int)(k0 - c) : 0;
    const int j1 = p.n - c < kWave ? (int)(p.n - c) : kWave;
#pragma unroll 1
    for (int j = j0; j < j1; ++j) {
      const float xc = lf_cls(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv), j)));
      lf_order();
      const float yc = cur[0] + b0 * xc;
      for (int i = lane; i < D; i += kWave) {
        const float up = i + 1 < D ? cur[i + 1] : 0.f;
        nxt[i] = up + lf_sign(p.b, i + 1) * xc - lf_sign(p.a, i + 1) * yc;
      }
      float* t = cur;
      cur = nxt;
      nxt = t;
      if (lane == j) ymine = yc;
    }
    if (kl >= k0 && kl < c + j1) y[kl] = ymine;
    // every state NaN: every later y is NaN
    lf_order();
    bool nan = true, same = true;
    for (int i = lane; i < D; i += kWave) {
      nan &= cur[i] != cur[i];
      same &= lf_same(cur[i], start[i]);
    }
    saturated = __ballot(!nan) == 0;
    // a whole chunk of finite x that returned the state to its start: the
    // labels are periodic with a period dividing kWave
    periodic = fin && j0 == 0 && j1 == kWave && __ballot(!same) == 0;
    yprev = ymine;
  }
  for (int64_t j = c + lane; j < p.n; j += kWave) y[j] = __builtin_nanf("");
}

}  // namespace

int launch_lfilter_nf(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x, int64_t ld_y,
                      const double* b, int nb, const double* a, int na, hipStream_t s) {
  DSP_REQUIRE(B >= 0 && n >= 0 && ld_x >= n && ld_y >= n, "bad sizes");
  DSP_REQUIRE(nb >= 1 && na >= 2, "lfilter repair needs len(b) >= 1 and len(a) >= 2 (len(a) == 1 "
                                  "is a convolution)");
  const int D = (na > nb ? na : nb) - 1;
  DSP_REQUIRE(D <= DSP_LFILTER_NF_MAX, "order %d above %d", D, DSP_LFILTER_NF_MAX);
  DSP_REQUIRE(b && a, "null coefficients");
  DSP_REQUIRE(a[0] != 0.0, "a[0] == 0");
  if (B == 0 || n == 0) return DSP_OK;
  DSP_REQUIRE(x && y, "null pointer");
  bool fir = true;  // a / a0 = [1, 0, ...]: the caller convolved (design.py 'fir_rec')
  for (int i = 1; i < na; ++i) fir &= a[i] == 0.0;
  LfNfArgs p{x, y, B, n, ld_x, ld_y, D, fir ? 1 : 0, {}, {}};
  auto put = [&](uint32_t* w, int i, const double* c, int nc) {
    const double q = i < nc ? c[i] / a[0] : 0.0;  // lfilter pads the shorter one with zeros
    w[i >> 4] |= (q > 0 ? 1u : (q < 0 ? 2u : 0u)) << (2 * (i & 15));
  };
  for (int i = 0; i <= D; ++i) {
    put(p.b, i, b, nb);
    put(p.a, i, a, na);
  }
  for (int64_t b0 = 0; b0 < B; b0 += 1 << 30) {
    LfNfArgs q = p;
    q.B = B - b0 < (1 << 30) ? B - b0 : (1 << 30);
    q.x = x + b0 * ld_x;
    q.y = y + b0 * ld_y;
    hipLaunchKernelGGL(k_lfilter_nf, dim3((unsigned)q.B), dim3(kWave), 3 * (size_t)D * sizeof(float),
                       s, q);
    DSP_LAUNCHED("k_lfilter_nf");
  }
  return DSP_OK;
}

}  // namespace dsp
