// Biquad-cascade realisation shared by the standalone cascade (iir.hip) and the
// single-pass chain kernel (chain_tile.hip).
//
// The reference filters with lfilter's direct form II transposed per band
// (modules/dsp_core.py:205-214, :233-254).  The kernels realise the same
// transfer functions in direct form II with the b0 gains pulled out (every
// b0 != 0, as for every EQ band):
//     u *= G = prod b0;  per stage:  w = u - a1 w1 - a2 w2
//                                    v = w + (b1/b0) w1 + (b2/b0) w2
// i.e. 4 fp64 FMAs per stage instead of DF2T's 4 FMAs + 1 multiply; with some
// b0 == 0 the stage keeps its gain (v = b0 w + b1 w1 + b2 w2, NORM = false).
// Both are exact rearrangements of one recursion and differ from lfilter by
// float64 rounding only.  The cascade is a D = 2S state linear system
// X' = A X + B u, state order (w1_0, w2_0, w1_1, w2_1, ...).
#pragma once

#include <cmath>
#include <vector>

#include "common.h"

namespace dsp {

// Direct form II realisation: c[k] = {g, c1, c2, a1, a2} and input gain G.
// NORM (every b0 != 0): g = 1, c1 = b1/b0, c2 = b2/b0, G = prod b0.
// Otherwise: g = b0, c1 = b1, c2 = b2, G = 1.  Stages past S are identities
// ({1, 0, 0, 0, 0}: w = u, v = w exactly).
struct SosParams {
  double c[DSP_MAX_STAGES][5];
  double G;
};

// Host: realisation of a [S][5] {b0 b1 b2 a1 a2} cascade; returns NORM.  Must
// match dspcore/design.py:df2_realization, which builds the state tables.
inline bool realize(const double* sos, int S, SosParams* p) {
  bool norm = true;
  for (int k = 0; k < S; ++k) norm = norm && sos[5 * k] != 0.0;
  p->G = 1.0;
  for (int k = 0; k < DSP_MAX_STAGES; ++k) {
    double* c = p->c[k];
    if (k >= S) {
      c[0] = 1.0;
      c[1] = c[2] = c[3] = c[4] = 0.0;
      continue;
    }
    const double* r = sos + 5 * k;
    if (norm) {
      c[0] = 1.0;
      c[1] = r[1] / r[0];
      c[2] = r[2] / r[0];
      p->G *= r[0];
    } else {
      c[0] = r[0];
      c[1] = r[1];
      c[2] = r[2];
    }
    c[3] = r[3];
    c[4] = r[4];
  }
  return norm;
}

// One sample through the S-stage cascade; w1/w2 are the stages' delay lines.
template <int S, bool NORM>
__device__ __forceinline__ double cascade_step(double u, double (&w1)[S > 0 ? S : 1],
                                               double (&w2)[S > 0 ? S : 1],
                                               const SosParams& p) {
  if constexpr (NORM && S > 0) u *= p.G;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const double w = fma(-p.c[k][4], w2[k], fma(-p.c[k][3], w1[k], u));
    const double h = NORM ? w : p.c[k][0] * w;
    u = fma(p.c[k][2], w2[k], fma(p.c[k][1], w1[k], h));
    w2[k] = w1[k];
    w1[k] = w;
  }
  return u;
}

// np.clip(v, lo, hi) with NaN kept: IEEE 754-2019 maximum/minimum propagate
// NaN (v_maximum3_f32 / v_minimum3_f32 on gfx950, two VALU).  Clipping after
// the float32 rounding gives the same result as rounding the float64 clip
// (|v| <= 1 rounds to |v| <= 1, anything beyond rounds to beyond-or-equal).
// lo/hi = -inf/+inf is the identity.
__device__ __forceinline__ float clip_f32(float v, float lo, float hi) {
  return __builtin_elementwise_minimum(__builtin_elementwise_maximum(v, lo), hi);
}

// One step of the realisation's state with input u: X <- A X + B u.  Host
// and device share it (columns of A with u = 0, B with X = 0 and u = 1).
__host__ __device__ inline void cascade_state_step(const SosParams& p, int S, bool norm,
                                                   double* X, double u) {
  if (norm) u *= p.G;
  for (int k = 0; k < S; ++k) {
    const double w = u - p.c[k][3] * X[2 * k] - p.c[k][4] * X[2 * k + 1];
    const double v = p.c[k][0] * w + p.c[k][1] * X[2 * k] + p.c[k][2] * X[2 * k + 1];
    X[2 * k + 1] = X[2 * k];
    X[2 * k] = w;
    u = v;
  }
}

// A of the D = 2S state system, float64, row-major.
inline std::vector<double> state_matrix(const SosParams& p, int S) {
  const int D = 2 * S;
  std::vector<double> A((size_t)D * D, 0.0);
  for (int col = 0; col < D; ++col) {
    std::vector<double> X(D, 0.0);
    X[col] = 1.0;
    cascade_state_step(p, S, false, X.data(), 0.0);
    for (int r = 0; r < D; ++r) A[(size_t)r * D + col] = X[r];
  }
  return A;
}

inline std::vector<double> matmul(const std::vector<double>& a, const std::vector<double>& b,
                                  int D) {
  std::vector<double> c((size_t)D * D, 0.0);
  for (int i = 0; i < D; ++i)
    for (int k = 0; k < D; ++k) {
      const double aik = a[(size_t)i * D + k];
      for (int j = 0; j < D; ++j)
        c[(size_t)i * D + j] = std::fma(aik, b[(size_t)k * D + j], c[(size_t)i * D + j]);
    }
  return c;
}

// A^T by square-and-multiply (the state transition across T samples).
inline std::vector<double> chunk_transition(const SosParams& p, int S, int64_t T) {
  const int D = 2 * S;
  std::vector<double> base = state_matrix(p, S), r((size_t)D * D, 0.0);
  for (int i = 0; i < D; ++i) r[(size_t)i * D + i] = 1.0;
  for (int64_t e = T; e > 0; e >>= 1) {
    if (e & 1) r = matmul(r, base, D);
    if (e > 1) base = matmul(base, base, D);
  }
  return r;
}

}  // namespace dsp
