// Polyphase L/M sample-rate converter for gfx950.
//
// Replaces reference modules/dsp_core.py:148-170: the expander (:149-150), the
// 'same' convolution with L*h (:162,:166) and the decimator (:170).  The
// reference computes N*L*K multiply-adds, (L-1)/L of them on inserted zeros,
// then drops (M-1)/M of the outputs.  Here only the kept outputs are computed
// and only the taps that meet a real input sample:
//
//   j = m*M + c, phi = j mod L, q = j div L
//   y[m] = sum_t P[phi][t] * x[q - t],  P[phi][t] = taps[phi + L*t]
//
// i.e. ceil(K/L) FMAs per output.  Both kernels stage the block's input window
// and the polyphase tap bank in LDS (coalesced, float4 where aligned) and
// stream the outputs back through LDS as float4 stores.  HBM traffic is the
// algorithmic minimum: x read once, y written once (window overlap between
// neighbouring blocks is T-1 samples out of thousands).
//
// The register-blocked kernel issues 752 VALU instructions per wave at config 3
// (profiles/r01_v8_pmc_summary).  DSP_SRC_PACK=1 accumulates taps u and u+1 of
// an output in the two halves of a v_pk_fma_f32 for even M (300 packed + 15
// scalar FMAs per thread instead of 615); measured 0.397 vs 0.398 ms on the same
// box, so the default build keeps the scalar chains (bitwise equal to the fused
// chain kernel's).  In chain mode 2 the same kernel also emits the cascade's
// chunk end states from the y tile it holds in LDS (emit_states, common.h
// SrcStates), which saves the cascade its first pass over the data.
#include "common.h"

#ifndef DSP_SRC_PACK
#define DSP_SRC_PACK 0  // 1: packed tap pairs (measured no faster on MI355X)
#endif

namespace dsp {
namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
// Constant address space: wave-uniform loads through it become scalar loads.
typedef const double __attribute__((address_space(4)))* const_f64_ptr;

// Fills win[i] = x[qa + i] for i < nload (zeros outside [0, n_in)).
// qa is a multiple of 4 so aligned rows allow float4 loads.
template <int NT>
__device__ __forceinline__ void load_window(float* __restrict__ win,
                                            const float* __restrict__ xr,
                                            int64_t qa, int nload, int64_t n_in,
                                            bool vec_ok) {
  const int nv = (nload + 3) >> 2;
  for (int v = threadIdx.x; v < nv; v += NT) {
    const int64_t q = qa + 4 * (int64_t)v;
    float4 f;
    if (vec_ok && q >= 0 && q + 3 < n_in) {
      f = *reinterpret_cast<const float4*>(xr + q);
    } else {
      f.x = (q + 0 >= 0 && q + 0 < n_in) ? xr[q + 0] : 0.f;
      f.y = (q + 1 >= 0 && q + 1 < n_in) ? xr[q + 1] : 0.f;
      f.z = (q + 2 >= 0 && q + 2 < n_in) ? xr[q + 2] : 0.f;
      f.w = (q + 3 >= 0 && q + 3 < n_in) ? xr[q + 3] : 0.f;
    }
    *reinterpret_cast<float4*>(win + 4 * v) = f;
  }
}

// Writes out[0:count] to yr[0:count] (float4 when the row is aligned).
template <int NT>
__device__ __forceinline__ void store_tile(float* __restrict__ yr,
                                           const float* __restrict__ out,
                                           int count, bool vec_ok) {
  if (vec_ok) {
    const int nv = count >> 2;
    for (int v = threadIdx.x; v < nv; v += NT)
      *reinterpret_cast<float4*>(yr + 4 * v) =
          *reinterpret_cast<const float4*>(out + 4 * v);
    for (int i = 4 * nv + threadIdx.x; i < count; i += NT) yr[i] = out[i];
  } else {
    for (int i = threadIdx.x; i < count; i += NT) yr[i] = out[i];
  }
}

// LDS slot of tile output l.  ST pads every kStU outputs with 4 floats so that
// emit_states' per-sub-chunk float4 reads (stride kStU + 4 floats) fall on 16
// distinct bank quads in every lane group of a ds_read_b128.
template <bool ST>
__device__ __forceinline__ int out_slot(int l) {
  if constexpr (ST) return l + 4 * (l / kStU);
  else return l;
}

// store_tile for the padded image.
template <int NT>
__device__ __forceinline__ void store_tile_padded(float* __restrict__ yr,
                                                  const float* __restrict__ out, int count,
                                                  bool vec_ok) {
  constexpr int V = kStU / 4;  // float4s per sub-chunk
  if (vec_ok) {
    const int nv = count >> 2;
    for (int v = threadIdx.x; v < nv; v += NT)
      *reinterpret_cast<float4*>(yr + 4 * v) =
          *reinterpret_cast<const float4*>(out + 4 * v + 4 * (v / V));
    for (int i = 4 * nv + threadIdx.x; i < count; i += NT) yr[i] = out[out_slot<true>(i)];
  } else {
    for (int i = threadIdx.x; i < count; i += NT) yr[i] = out[out_slot<true>(i)];
  }
}

// Chain mode 2: the cascade's chunk end states from this block's y tile
// (common.h SrcStates), in two steps:
//  1. sub-chunk j (kStU outputs) from zero state: s_j = sum_t g[t] y[t], lane j
//     of each wave, wave w computing components 4w..4w+3 (g through scalar
//     loads: the address is wave-uniform);
//  2. every chunk piece in the tile carried to its chunk's end by Horner steps
//     S <- A^kStU S + s_j (zero input past the tile), lane (piece, row i)
//     holding row i of A^kStU in registers and S in LDS; the 16 lanes of a
//     piece sit in one wave, whose LDS operations execute in order (no barrier).
// The y values are the float32 outputs exactly as stored, so the states are the
// ones the cascade's own first pass would compute, up to float64 summation order.
template <int TILE, int NT>
__device__ __forceinline__ void emit_states(const float* s_out, double* scratch,
                                            const SrcStates& st, int64_t b, int64_t m0) {
  constexpr int NSUB = TILE / kStU, D = kStD;
  static_assert(NSUB <= kWave && NT == 3 * kWave && D == 12, "3 waves x 4 state components");
  static_assert(NT / 16 == kStPieces, "16 lanes per chunk piece");
  const int tid = threadIdx.x;
  double* sst = scratch;            // [NSUB][D] sub-chunk states
  double* hs = scratch + NSUB * D;  // [kStPieces][D] Horner states
  {
    const int j = tid & (kWave - 1);
    const int grp = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifndef DSP_ST_EXP
#define DSP_ST_EXP 0  // timing ablations: 1 no sub-chunk dot products, 2 no Horner steps
#endif
    if (j < NSUB && DSP_ST_EXP != 1) {
      const float* yy = s_out + j * (kStU + 4);
      const const_f64_ptr g = (const_f64_ptr)st.g + 4 * grp;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll 4
      for (int t4 = 0; t4 < kStU; t4 += 4) {
        const float4 v = *reinterpret_cast<const float4*>(yy + t4);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double u = (double)vv[e];
          const const_f64_ptr gt = g + (t4 + e) * D;
          a0 = fma(gt[0], u, a0);
          a1 = fma(gt[1], u, a1);
          a2 = fma(gt[2], u, a2);
          a3 = fma(gt[3], u, a3);
        }
      }
      double* d = sst + j * D + 4 * grp;
      d[0] = a0;
      d[1] = a1;
      d[2] = a2;
      d[3] = a3;
    }
  }
  lds_barrier();  // LDS only: the tile's y stores stay in flight
  const int pc = tid >> 4, i = tid & 15;
  const int64_t Tc = st.chunk_len;
  const int NJ = (int)(Tc / kStU);
  const int64_t jt0 = m0 / kStU;    // the tile's first sub-chunk
  const int64_t ck = m0 / Tc + pc;  // this piece's chunk
  const bool act = i < D && ck + 1 < st.C && ck * Tc < m0 + TILE;
  const int64_t cs = ck * NJ;       // the chunk's first sub-chunk
  const int ja = (int)(max(cs, jt0) - jt0);
  const int jb = (int)min((int64_t)NSUB, cs + NJ - jt0);
  const int steps = act && DSP_ST_EXP != 2 ? (int)(cs + NJ - jt0) - ja : 0;
  const int ir = i < D ? i : 0;
  double arow[D];
#pragma unroll
  for (int m = 0; m < D; ++m) arow[m] = st.AU[ir * D + m];
  double* h = hs + pc * D;
  double acc = 0.0;
  if (act) h[i] = 0.0;
  asm volatile("" ::: "memory");
  for (int s = 0; s < NJ; ++s) {
    if (s < steps) {
      const int jl = ja + s;
      double p0 = jl < jb ? sst[jl * D + i] : 0.0, p1 = 0.0, p2 = 0.0;
#pragma unroll
      for (int m = 0; m < D; m += 3) {
        p0 = fma(arow[m], h[m], p0);
        p1 = fma(arow[m + 1], h[m + 1], p1);
        p2 = fma(arow[m + 2], h[m + 2], p2);
      }
      acc = (p0 + p1) + p2;
    }
    asm volatile("" ::: "memory");  // every lane's reads of S precede the writes
    if (s < steps) h[i] = acc;
    asm volatile("" ::: "memory");
  }
  if (act) {
    const int64_t slot = m0 / TILE - ck * Tc / TILE;
    st.part[((b * st.C + ck) * 2 + slot) * D + i] = acc;
  }
}

// ---------------------------------------------------------------------------
// Register-blocked kernel for a compile-time (L, M, T).
// Thread (p, g) owns the R outputs m = m0 + p + g*L*R + r*L, r < R.  They share
// one polyphase branch phi, and their input windows are shifted by M samples,
// so one tap read feeds R FMAs and one window read feeds up to T FMAs:
// (T + (R-1)M) + T LDS reads per R*T FMAs.  ST: chain mode 2 (emit_states).
// ---------------------------------------------------------------------------
template <int L, int M, int T, int R, int NT, bool ST>
__global__ __launch_bounds__(NT) void k_src_reg(
    const float* __restrict__ x, float* __restrict__ y, int64_t n_in,
    int64_t ld_x, int64_t n_out, int64_t ld_y, const float* __restrict__ taps,
    int K, int64_t c, int vec_x, int vec_y, SrcStates st) {
  constexpr int G = NT / L;          // thread groups with one thread per phase
  constexpr int TILE = G * L * R;    // outputs per block
  constexpr int TP = ((T + 3) / 4) * 4 + 4;               // padded bank row
  constexpr int WMAX = ((TILE - 1) * M) / L + T + 2 + 8;  // window + align slack
  constexpr int WF = ((WMAX + 3) / 4) * 4;
  constexpr int OUTF = ST ? TILE + 4 * (TILE / kStU) : TILE;
  static_assert(TILE % 4 == 0, "tile must be float4 aligned");
  static_assert(!ST || (TILE % kStU == 0 && (TILE / kStU + kStPieces) * kStD * 2 <= WF),
                "state emission: whole sub-chunks per tile, scratch inside the window");

  __shared__ __attribute__((aligned(16))) float s_bank[L * TP];
  __shared__ __attribute__((aligned(16))) float s_win[WF];
  __shared__ __attribute__((aligned(16))) float s_out[OUTF];

  const int tid = threadIdx.x;
  const int64_t b = blockIdx.y;
  const int64_t m0 = (int64_t)blockIdx.x * TILE;
  const float* xr = x + b * ld_x;
  float* yr = y + b * ld_y;

  const int64_t qlo = (m0 * M + c) / L - (T - 1);
  const int64_t qhi = ((m0 + TILE - 1) * M + c) / L;
  const int64_t qa = qlo & ~(int64_t)3;
  load_window<NT>(s_win, xr, qa, (int)(qhi - qa + 1), n_in, vec_x != 0);

  // Bank row phi holds the branch taps reversed: s_bank[phi][u] = P[phi][T-1-u].
  for (int i = tid; i < L * TP; i += NT) {
    const int phi = i / TP, u = i - phi * TP;
    const int k = phi + L * (T - 1 - u);
    s_bank[i] = (u < T && k < K) ? taps[k] : 0.f;
  }
  __syncthreads();

  if (tid < G * L) {
    const int p = tid % L, g = tid / L;
    const int lbase = p + g * L * R;                 // local index of r = 0
    const int64_t j = (m0 + lbase) * M + c;
    const int64_t q = j / L;
    const int phi = (int)(j - q * L);
    const float* w = s_win + (int)(q - (T - 1) - qa);
    const float* h = s_bank + phi * TP;
    float acc[R];
    if constexpr (DSP_SRC_PACK && M % 2 == 0) {
      // Taps u, u+1 in the two halves of a v_pk_fma_f32.  With M even every
      // window pair (w[r*M + u], w[r*M + u + 1]) starts at an even offset, so
      // each pair is loaded once and feeds up to R outputs.
      f32x2 a2[R];
#pragma unroll
      for (int r = 0; r < R; ++r) a2[r] = f32x2{0.f, 0.f};
#pragma unroll
      for (int u = 0; u + 1 < T; u += 2) {
        const f32x2 t2 = *reinterpret_cast<const f32x2*>(h + u);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const f32x2 wv = {w[r * M + u], w[r * M + u + 1]};
          a2[r] = __builtin_elementwise_fma(t2, wv, a2[r]);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float e = a2[r].x;
        if constexpr (T % 2 == 1) e = fmaf(h[T - 1], w[r * M + T - 1], e);
        acc[r] = e + a2[r].y;
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = 0.f;
#pragma unroll
      for (int u = 0; u < T; ++u) {
        const float t = h[u];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = fmaf(t, w[r * M + u], acc[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) s_out[out_slot<ST>(lbase + r * L)] = acc[r];
  }
  __syncthreads();

  const int64_t count = min((int64_t)TILE, n_out - m0);
  if constexpr (ST) {
    store_tile_padded<NT>(yr + m0, s_out, (int)count, vec_y != 0);
    emit_states<TILE, NT>(s_out, reinterpret_cast<double*>(s_win), st, b, m0);
  } else {
    store_tile<NT>(yr + m0, s_out, (int)count, vec_y != 0);
  }
}

// ---------------------------------------------------------------------------
// Generic kernel: any L, M, K.  One output per thread-iteration, T taps each.
// LDS: tap bank [L][T] + input window, both carved from dynamic LDS.
// ---------------------------------------------------------------------------
constexpr int kGenNT = 256;
constexpr int kGenTile = 4096;

__global__ __launch_bounds__(kGenNT) void k_src_generic(
    const float* __restrict__ x, float* __restrict__ y, int64_t n_in,
    int64_t ld_x, int64_t n_out, int64_t ld_y, const float* __restrict__ taps,
    int K, int L, int M, int T, int64_t c, int tile, int bank_floats,
    int vec_x, int vec_y) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_bank = smem;                       // [L][T], bank_floats (mult. of 4)
  float* s_win = smem + bank_floats;          // window
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.y;
  const int64_t m0 = (int64_t)blockIdx.x * tile;
  const int64_t m1 = min(m0 + tile, n_out);
  const float* xr = x + b * ld_x;
  float* yr = y + b * ld_y;

  const int64_t qlo = (m0 * M + c) / L - (T - 1);
  const int64_t qhi = ((m1 - 1) * M + c) / L;
  const int64_t qa = qlo & ~(int64_t)3;
  load_window<kGenNT>(s_win, xr, qa, (int)(qhi - qa + 1), n_in, vec_x != 0);
  for (int i = tid; i < L * T; i += kGenNT) {
    const int phi = i / T, u = i - phi * T;
    const int k = phi + L * (T - 1 - u);
    s_bank[i] = (k < K) ? taps[k] : 0.f;
  }
  __syncthreads();

  // Output stores are coalesced directly (consecutive threads, consecutive m).
  // (q, phi) of j = m*M + c advance by a fixed (dq, dphi) per iteration, so the
  // 64-bit division happens once per thread.
  (void)vec_y;
  const int64_t j0 = (m0 + tid) * M + c;
  int64_t q = j0 / L;
  int phi = (int)(j0 - q * L);
  const int64_t step = (int64_t)kGenNT * M;
  const int64_t dq = step / L;
  const int dphi = (int)(step - dq * L);
  for (int64_t m = m0 + tid; m < m1; m += kGenNT) {
    const float* w = s_win + (int)(q - (T - 1) - qa);
    const float* h = s_bank + phi * T;
    float a0 = 0.f, a1 = 0.f;
    int u = 0;
    for (; u + 1 < T; u += 2) {
      a0 = fmaf(h[u], w[u], a0);
      a1 = fmaf(h[u + 1], w[u + 1], a1);
    }
    if (u < T) a0 = fmaf(h[u], w[u], a0);
    yr[m] = a0 + a1;
    q += dq;
    phi += dphi;
    if (phi >= L) {
      phi -= L;
      ++q;
    }
  }
}

template <int L, int M, int T, int R, int NT, bool ST = false>
int run_reg(const float* x, float* y, int64_t B, int64_t n_in, int64_t ld_x,
            int64_t n_out, int64_t ld_y, const float* taps, int K, int64_t c,
            int vec_x, int vec_y, const SrcStates& st, hipStream_t s) {
  constexpr int TILE = (NT / L) * L * R;
  dim3 grid((unsigned)ceil_div(n_out, TILE), (unsigned)B);
  TraceScope trace(ST ? "src_states" : "src_poly", s);
  hipLaunchKernelGGL((k_src_reg<L, M, T, R, NT, ST>), grid, dim3(NT), 0, s, x, y,
                     n_in, ld_x, n_out, ld_y, taps, K, c, vec_x, vec_y, st);
  DSP_LAUNCHED("k_src_reg");
  return DSP_OK;
}

// TILE of run_reg<3, 2, 41, 15, 192>, the instantiation that emits states.
constexpr int kStTile = (192 / 3) * 3 * 15;

}  // namespace

int src_states_tile(int L, int M, int K) {
  return (L == 3 && M == 2 && (K + L - 1) / L == 41) ? kStTile : 0;
}

int launch_src_states(const float* x, float* y, int64_t B, int64_t n_in, int64_t ld_x,
                      int64_t n_out, int64_t ld_y, const float* taps, int K, int L, int M,
                      int64_t c, const SrcStates& st, hipStream_t s) {
  if (!src_states_tile(L, M, K)) return kNotFused;
  DSP_REQUIRE(B >= 0 && n_in >= 1 && n_out >= 0 && c >= 0, "bad sizes B=%lld n_in=%lld",
              (long long)B, (long long)n_in);
  DSP_REQUIRE(ld_x >= n_in && ld_y >= n_out, "leading dimension too small");
  DSP_REQUIRE(B <= 65535, "B=%lld exceeds the grid's y extent (65535); split the batch",
              (long long)B);
  DSP_REQUIRE(st.chunk_len > 0 && st.chunk_len % kStU == 0 && st.chunk_len <= kStTile &&
                  ceil_div(kStTile - 1, st.chunk_len) + 1 <= kStPieces &&
                  st.C == ceil_div(n_out, st.chunk_len),
              "chunk_len=%lld does not fit the SRC's state emission", (long long)st.chunk_len);
  if (B == 0 || n_out == 0) return DSP_OK;
  DSP_REQUIRE(x && y && taps && st.part && st.g, "null pointer");
  const int vec_x = ((ld_x & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0);
  const int vec_y = ((ld_y & 3) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0);
  return run_reg<3, 2, 41, 15, 192, true>(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, c, vec_x,
                                          vec_y, st, s);
}

int launch_src(const float* x, float* y, int64_t B, int64_t n_in, int64_t ld_x,
               int64_t n_out, int64_t ld_y, const float* taps, int K, int L,
               int M, int64_t c, hipStream_t s) {
  DSP_REQUIRE(B >= 0 && n_in >= 1 && n_out >= 0, "bad sizes B=%lld n_in=%lld n_out=%lld",
              (long long)B, (long long)n_in, (long long)n_out);
  DSP_REQUIRE(L >= 1 && M >= 1 && K >= 1, "bad L=%d M=%d K=%d", L, M, K);
  DSP_REQUIRE(c >= 0, "bad c_offset %lld", (long long)c);
  DSP_REQUIRE(ld_x >= n_in && ld_y >= n_out, "leading dimension too small");
  DSP_REQUIRE(B <= 65535, "B=%lld exceeds the grid's y extent (65535); split the batch",
              (long long)B);
  if (B == 0 || n_out == 0) return DSP_OK;
  DSP_REQUIRE(x && y && taps, "null pointer");
  const int T = (K + L - 1) / L;
  const int vec_x = ((ld_x & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0);
  const int vec_y = ((ld_y & 3) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0);

  // Register-blocked instantiations: the benchmark configurations and the
  // app's most common (L, M) pairs with the default tap rule 40*max(L,M)+1.
  // R is chosen so that R*M is not a multiple of 32: thread groups' windows
  // start R*M floats apart and must land on different LDS banks.
  const SrcStates none{};
  if (L == 3 && M == 2 && T == 41)
    return run_reg<3, 2, 41, 15, 192>(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, c, vec_x, vec_y,
                                      none, s);
  if (L == 3 && M == 2 && T == 85)
    return run_reg<3, 2, 85, 7, 192>(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, c, vec_x, vec_y,
                                     none, s);
  if (L == 2 && M == 1 && T == 64)
    return run_reg<2, 1, 64, 15, 256>(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, c, vec_x, vec_y,
                                      none, s);
  if (L == 2 && M == 1 && T == 41)
    return run_reg<2, 1, 41, 15, 256>(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, c, vec_x, vec_y,
                                      none, s);

  // Generic path.  Shrink the tile until bank + window fit in LDS.
  const int bank_floats = ((L * T + 3) / 4) * 4;
  int tile = kGenTile;
  auto lds_bytes = [&](int t) {
    const int64_t w = ((int64_t)(t - 1) * M) / L + T + 2 + 8;
    return (int64_t)(bank_floats + ((w + 3) / 4) * 4) * 4;
  };
  while (tile > 64 && lds_bytes(tile) > 160 * 1024) tile >>= 1;
  if (lds_bytes(tile) > 160 * 1024)
    return set_error(DSP_ENOTSUP, "tap bank L*ceil(K/L)=%d floats does not fit in LDS", L * T);
  dim3 grid((unsigned)ceil_div(n_out, tile), (unsigned)B);
  const size_t shm = (size_t)lds_bytes(tile);
  if (int rc = allow_lds(k_src_generic, shm)) return rc;
  TraceScope trace("src_poly", s);
  hipLaunchKernelGGL(k_src_generic, grid, dim3(kGenNT), shm, s, x, y, n_in, ld_x,
                     n_out, ld_y, taps, K, L, M, T, c, tile, bank_floats, vec_x, vec_y);
  DSP_LAUNCHED("k_src_generic");
  return DSP_OK;
}

}  // namespace dsp
