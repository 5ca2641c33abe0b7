// Biquad cascade (DF2T) for gfx950, float64 arithmetic, float32 I/O.
//
// Replaces reference modules/dsp_core.py:233-254: the serial loop of
// aplicar_ecuacion_diferencias (= scipy.signal.lfilter(b, a, x), :205-214) over
// the EQ bands followed by np.clip(y, -1, 1) (:254).  lfilter realises each
// biquad in direct form II transposed with zero initial state:
//     v = b0 u + s1;  s1 = b1 u - a1 v + s2;  s2 = b2 u - a2 v
// Float64 state and coefficients are mandatory: the 40 Hz band has poles at
// |r| = 0.99926 and a float32 recursion drifts by ~1e-3.
//
// The recursion is serial in time, and one lane per channel leaves the chip
// ~16x under-filled at 4096 channels.  The S-stage cascade is a 2S-state
// linear system X' = A X + B u, so the time axis is cut into chunks of T
// samples and the exact chunk initial states are recovered with a carry scan:
//   pass 1 (k_iir_pass<S,false>): run every chunk but the last from zero state,
//          keep its end state E_c                               (lanes = B*(C-1))
//   carry  (k_iir_carry):  S_0 = 0,  S_{c+1} = A^T S_c + E_c    (lanes = B)
//   pass 2 (k_iir_pass<S,true>):  rerun every chunk from S_c, clip, store
// A^T is built on the device from the coefficients (k_iir_prep).  The chunk
// length depends only on the caller's chunk_len, never on B, so a batch gives
// bitwise-identical rows however it is sharded over GPUs.
//
// Memory: lanes are (channel, chunk) rows; a 256-row x 32-sample tile is
// loaded with coalesced 128-byte row segments into LDS (row stride 33 floats:
// conflict-free per-lane column reads), each lane walks its row, and pass 2
// writes its outputs back into the same tile before a coalesced store.
#include "common.h"

namespace dsp {
namespace {

struct SosParams {
  double c[DSP_MAX_STAGES][5];  // b0 b1 b2 a1 a2
};

constexpr int kIirNT = 256;
constexpr int kTS = 32;        // samples per tile step
constexpr int kRow = kTS + 1;  // LDS row stride in floats

template <int S>
__device__ __forceinline__ double cascade_step(double u, double (&s1)[S > 0 ? S : 1],
                                               double (&s2)[S > 0 ? S : 1],
                                               const SosParams& p) {
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const double v = fma(p.c[k][0], u, s1[k]);
    s1[k] = fma(-p.c[k][3], v, fma(p.c[k][1], u, s2[k]));
    s2[k] = fma(-p.c[k][4], v, p.c[k][2] * u);
    u = v;
  }
  return u;
}

__device__ __forceinline__ double clip1(double v) {
  // np.clip semantics: NaN stays NaN.
  return v < -1.0 ? -1.0 : (v > 1.0 ? 1.0 : v);
}

// APPLY = false: pass 1 (end states of chunks 0..C-2, zero initial state).
// APPLY = true : pass 2 (all C chunks from their carried initial state).
template <int S, bool APPLY>
__global__ __launch_bounds__(kIirNT) void k_iir_pass(
    const float* __restrict__ x, float* __restrict__ y, int64_t n,
    int64_t ld_x, int64_t ld_y, SosParams p, int64_t C, int64_t T,
    int64_t lanes, const double* __restrict__ s_init, double* __restrict__ e_out,
    int clip, int vec_x, int vec_y) {
  constexpr int SS = S > 0 ? S : 1;
  __shared__ __attribute__((aligned(16))) float tile[kIirNT * kRow];
  __shared__ int64_t row_in[kIirNT];
  __shared__ int64_t row_out[kIirNT];
  __shared__ int row_len[kIirNT];

  const int tid = threadIdx.x;
  const int64_t g = (int64_t)blockIdx.x * kIirNT + tid;
  const int64_t cl = APPLY ? C : C - 1;  // chunks per channel handled here
  const bool live = g < lanes;
  int64_t b = 0, ch = 0;
  if (live) {
    b = g / cl;
    ch = g - b * cl;
  }
  const int64_t t_begin = ch * T;
  row_in[tid] = b * ld_x + t_begin;
  row_out[tid] = b * ld_y + t_begin;
  row_len[tid] = live ? (int)min(T, n - t_begin) : 0;

  double s1[SS], s2[SS];
#pragma unroll
  for (int k = 0; k < SS; ++k) s1[k] = s2[k] = 0.0;
  if (APPLY && live && ch > 0) {
    const double* si = s_init + (b * C + ch) * (2 * S);
#pragma unroll
    for (int k = 0; k < S; ++k) {
      s1[k] = si[2 * k];
      s2[k] = si[2 * k + 1];
    }
  }
  __syncthreads();

  float* my = tile + tid * kRow;
  for (int64_t t0 = 0; t0 < T; t0 += kTS) {
    // Coalesced load: 8 threads x float4 per 128-byte row segment.
#pragma unroll
    for (int i = 0; i < (kIirNT * kTS / 4) / kIirNT; ++i) {
      const int f = i * kIirNT + tid;
      const int r = f >> 3, c4 = (f & 7) * 4;
      const int len = row_len[r];
      const int64_t t = t0 + c4;
      const float* src = x + row_in[r] + t;
      float4 v;
      if (vec_x && t + 3 < len) {
        v = *reinterpret_cast<const float4*>(src);
      } else {
        v.x = (t + 0 < len) ? src[0] : 0.f;
        v.y = (t + 1 < len) ? src[1] : 0.f;
        v.z = (t + 2 < len) ? src[2] : 0.f;
        v.w = (t + 3 < len) ? src[3] : 0.f;
      }
      float* d = tile + r * kRow + c4;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
    __syncthreads();

    // Samples past the end of a (last, partial) chunk are zeros; their
    // outputs are never stored and that lane's final state is never used.
#pragma unroll 8
    for (int j = 0; j < kTS; ++j) {
      double v = cascade_step<S>((double)my[j], s1, s2, p);
      if (APPLY) my[j] = (float)(clip ? clip1(v) : v);
    }

    if (APPLY) {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < (kIirNT * kTS / 4) / kIirNT; ++i) {
        const int f = i * kIirNT + tid;
        const int r = f >> 3, c4 = (f & 7) * 4;
        const int len = row_len[r];
        const int64_t t = t0 + c4;
        float* dst = y + row_out[r] + t;
        const float* s = tile + r * kRow + c4;
        if (vec_y && t + 3 < len) {
          *reinterpret_cast<float4*>(dst) = make_float4(s[0], s[1], s[2], s[3]);
        } else {
          if (t + 0 < len) dst[0] = s[0];
          if (t + 1 < len) dst[1] = s[1];
          if (t + 2 < len) dst[2] = s[2];
          if (t + 3 < len) dst[3] = s[3];
        }
      }
    }
    __syncthreads();
  }

  if (!APPLY && live) {
    double* e = e_out + g * (2 * S);
#pragma unroll
    for (int k = 0; k < S; ++k) {
      e[2 * k] = s1[k];
      e[2 * k + 1] = s2[k];
    }
  }
}

// One lane per channel: S_0 = 0, S_{c+1} = P S_c + E_c, P = A^T (D x D).
// The state vectors live in LDS ([D][256] doubles, double-buffered) so the
// kernel stays small for every D; it is a few microseconds of serial work.
template <int S>
__global__ __launch_bounds__(256) void k_iir_carry(const double* __restrict__ P,
                                                   const double* __restrict__ E,
                                                   double* __restrict__ s_init,
                                                   int64_t B, int64_t C) {
  constexpr int D = 2 * S;
  __shared__ double sP[D * D];
  __shared__ double st[2][D][256];
  const int tid = threadIdx.x;
  for (int i = tid; i < D * D; i += blockDim.x) sP[i] = P[i];
  for (int i = 0; i < D; ++i) st[0][i][tid] = 0.0;
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + tid;
  if (b >= B) return;
  int cur = 0;
  for (int64_t ch = 1; ch < C; ++ch) {
    const double* e = E + (b * (C - 1) + (ch - 1)) * D;
    double* o = s_init + (b * C + ch) * D;
    for (int i = 0; i < D; ++i) {
      double a = e[i];
#pragma unroll 4
      for (int j = 0; j < D; ++j) a = fma(sP[i * D + j], st[cur][j][tid], a);
      st[cur ^ 1][i][tid] = a;
      o[i] = a;
    }
    cur ^= 1;
  }
}

// Builds A (one cascade step on each unit state, zero input) and P = A^T by
// square-and-multiply, all in float64 inside one workgroup.
__global__ __launch_bounds__(1024) void k_iir_prep(SosParams p, int S, int64_t T,
                                                  double* __restrict__ P_out) {
  __shared__ double sA[32 * 32], sR[32 * 32], sTmp[32 * 32];
  const int D = 2 * S;
  const int tid = threadIdx.x;
  if (tid < D) {
    // state vector e_tid: s1_k = X[2k], s2_k = X[2k+1]
    double X[32];
    for (int i = 0; i < D; ++i) X[i] = (i == tid) ? 1.0 : 0.0;
    double u = 0.0;
    for (int k = 0; k < S; ++k) {
      const double v = p.c[k][0] * u + X[2 * k];
      const double n1 = p.c[k][1] * u - p.c[k][3] * v + X[2 * k + 1];
      const double n2 = p.c[k][2] * u - p.c[k][4] * v;
      X[2 * k] = n1;
      X[2 * k + 1] = n2;
      u = v;
    }
    for (int i = 0; i < D; ++i) sA[i * D + tid] = X[i];
  }
  const int r = tid / 32, c = tid % 32;
  if (r < D && c < D) sR[r * D + c] = (r == c) ? 1.0 : 0.0;
  __syncthreads();
  for (int64_t e = T; e > 0; e >>= 1) {
    if (e & 1) {  // R = R * A
      double a = 0.0;
      if (r < D && c < D)
        for (int k = 0; k < D; ++k) a = fma(sR[r * D + k], sA[k * D + c], a);
      __syncthreads();
      if (r < D && c < D) sR[r * D + c] = a;
      __syncthreads();
    }
    {  // A = A * A
      double a = 0.0;
      if (r < D && c < D)
        for (int k = 0; k < D; ++k) a = fma(sA[r * D + k], sA[k * D + c], a);
      __syncthreads();
      if (r < D && c < D) sTmp[r * D + c] = a;
      __syncthreads();
      if (r < D && c < D) sA[r * D + c] = sTmp[r * D + c];
      __syncthreads();
    }
  }
  if (r < D && c < D) P_out[r * D + c] = sR[r * D + c];
}

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

struct WsLayout {
  size_t p_off, e_off, s_off, total;
};

WsLayout ws_layout(int64_t B, int64_t n, int S, int64_t T) {
  WsLayout w{0, 0, 0, 0};
  const int64_t C = (S == 0 || T <= 0) ? 1 : ceil_div(n, T);
  if (C <= 1) return w;
  const size_t D = 2 * (size_t)S;
  w.p_off = 0;
  w.e_off = align256(D * D * sizeof(double));
  w.s_off = w.e_off + align256((size_t)B * (C - 1) * D * sizeof(double));
  w.total = w.s_off + align256((size_t)B * C * D * sizeof(double));
  return w;
}

template <int S>
int run_cascade(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x,
                int64_t ld_y, const SosParams& p, int clip, int64_t T, void* ws,
                hipStream_t s) {
  const int vec_x = ((ld_x & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0);
  const int vec_y = ((ld_y & 3) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0);
  const int64_t C = (S == 0) ? 1 : ceil_div(n, T);
  if (C == 1) T = ceil_div(n, kTS) * kTS;
  const WsLayout w = ws_layout(B, n, S, T);
  char* base = static_cast<char*>(ws);
  double* P = reinterpret_cast<double*>(base + w.p_off);
  double* E = reinterpret_cast<double*>(base + w.e_off);
  double* SI = reinterpret_cast<double*>(base + w.s_off);
  if (C > 1) {
    {
    TraceScope trace("iir_prep", s);
    hipLaunchKernelGGL(k_iir_prep, dim3(1), dim3(1024), 0, s, p, S, T, P);
    }
    DSP_LAUNCHED("k_iir_prep");
    const int64_t lanes1 = B * (C - 1);
    {
    TraceScope trace("iir_state", s);
    hipLaunchKernelGGL((k_iir_pass<S, false>), dim3((unsigned)ceil_div(lanes1, kIirNT)),
                       dim3(kIirNT), 0, s, x, y, n, ld_x, ld_y, p, C, T, lanes1,
                       (const double*)nullptr, E, clip, vec_x, vec_y);
    }
    DSP_LAUNCHED("k_iir_pass<state>");
    {
    TraceScope trace("iir_carry", s);
    hipLaunchKernelGGL((k_iir_carry<(S > 0 ? S : 1)>), dim3((unsigned)ceil_div(B, 256)),
                       dim3(256), 0, s, P, E, SI, B, C);
    }
    DSP_LAUNCHED("k_iir_carry");
  }
  const int64_t lanes2 = B * C;
  {
  TraceScope trace("iir_apply", s);
  hipLaunchKernelGGL((k_iir_pass<S, true>), dim3((unsigned)ceil_div(lanes2, kIirNT)),
                     dim3(kIirNT), 0, s, x, y, n, ld_x, ld_y, p, C, T, lanes2,
                     SI, (double*)nullptr, clip, vec_x, vec_y);
  }
  DSP_LAUNCHED("k_iir_pass<apply>");
  return DSP_OK;
}

}  // namespace

size_t biquad_workspace_bytes(int64_t B, int64_t n, int S, int64_t chunk_len) {
  if (B <= 0 || n <= 0 || S < 0 || S > DSP_MAX_STAGES || chunk_len <= 0) return 0;
  int Sp = S;
  if (S == 7) Sp = 8;
  else if (S > 8 && S <= 12) Sp = 12;
  else if (S > 12) Sp = 16;
  return ws_layout(B, n, Sp, chunk_len).total;
}

int launch_biquad(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x,
                  int64_t ld_y, const double* sos, int S, int clip,
                  int64_t chunk_len, void* ws, size_t ws_bytes, hipStream_t s) {
  DSP_REQUIRE(B >= 0 && n >= 0, "bad sizes");
  DSP_REQUIRE(S >= 0 && S <= DSP_MAX_STAGES, "S=%d outside [0, %d]", S, DSP_MAX_STAGES);
  DSP_REQUIRE(chunk_len > 0 && chunk_len % kTS == 0,
              "chunk_len=%lld must be a positive multiple of %d", (long long)chunk_len, kTS);
  DSP_REQUIRE(ld_x >= n && ld_y >= n, "leading dimension too small");
  if (B == 0 || n == 0) return DSP_OK;
  DSP_REQUIRE(x && y, "null pointer");
  DSP_REQUIRE(S == 0 || sos, "null sos");
  // Pad S up to an instantiated size with exact identity stages (b = 1,0,0; a = 0,0).
  int Sp = S;
  if (S == 7) Sp = 8;
  else if (S > 8 && S <= 12) Sp = 12;
  else if (S > 12) Sp = 16;
  SosParams p;
  for (int k = 0; k < DSP_MAX_STAGES; ++k) {
    for (int i = 0; i < 5; ++i) p.c[k][i] = (k < S) ? sos[5 * k + i] : (i == 0 ? 1.0 : 0.0);
  }
  const size_t need = ws_layout(B, n, Sp, chunk_len).total;
  DSP_REQUIRE(ws_bytes >= need, "workspace too small: %zu < %zu bytes", ws_bytes, need);
  DSP_REQUIRE(need == 0 || ws, "null workspace");
  switch (Sp) {
    case 0: return run_cascade<0>(x, y, B, n, ld_x, ld_y, p, clip, chunk_len, ws, s);
    case 1: return run_cascade<1>(x, y, B, n, ld_x, ld_y, p, clip, chunk_len, ws, s);
    case 2: return run_cascade<2>(x, y, B, n, ld_x, ld_y, p, clip, chunk_len, ws, s);
    case 3: return run_cascade<3>(x, y, B, n, ld_x, ld_y, p, clip, chunk_len, ws, s);
    case 4: return run_cascade<4>(x, y, B, n, ld_x, ld_y, p, clip, chunk_len, ws, s);
    case 5: return run_cascade<5>(x, y, B, n, ld_x, ld_y, p, clip, chunk_len, ws, s);
    case 6: return run_cascade<6>(x, y, B, n, ld_x, ld_y, p, clip, chunk_len, ws, s);
    case 8: return run_cascade<8>(x, y, B, n, ld_x, ld_y, p, clip, chunk_len, ws, s);
    case 12: return run_cascade<12>(x, y, B, n, ld_x, ld_y, p, clip, chunk_len, ws, s);
    case 16: return run_cascade<16>(x, y, B, n, ld_x, ld_y, p, clip, chunk_len, ws, s);
    default: return set_error(DSP_EINVAL, "unsupported stage count %d", S);
  }
}

}  // namespace dsp
