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
// The register-blocked kernel is the standalone SRC and the two-launch chain's
// first kernel; the chain's default path computes the same outputs inside its
// single-pass kernel (chain_tile.hip), in the same summation order.
#include "common.h"

namespace dsp {
namespace {

// Fills win[i] = x[qa + i] for i < nload (zeros outside [0, n_in)).
// qa is a multiple of 4 so aligned rows allow float4 loads.  Returns whether
// this thread loaded an inf or NaN (nf_acc).
template <int NT>
__device__ __forceinline__ bool load_window(float* __restrict__ win,
                                            const float* __restrict__ xr,
                                            int64_t qa, int nload, int64_t n_in,
                                            bool vec_ok) {
  nf_f32x2 nf = {0.f, 0.f};
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
    nf = nf_acc(nf, f);
  }
  return nf_any(nf);
}

// Flush threshold of the caller's taps (common.h, kTapFlushRel) for a block of
// NT threads: the same float32 max and product as tap_flush_threshold, so the
// device-staged tap banks flush exactly the taps the host tables do.  red:
// NT / 64 floats of LDS.  Contains a barrier.
template <int NT>
__device__ __forceinline__ float block_flush_threshold(const float* __restrict__ taps, int K, int L,
                                                       float* red) {
  if (L <= 1) return -1.f;
  float m = 0.f;
  for (int k = threadIdx.x; k < K; k += NT) m = fmaxf(m, fabsf(taps[k]));
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) r = fmaxf(r, red[w]);
  return kTapFlushRel * r;
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

// ---------------------------------------------------------------------------
// Register-blocked kernel for a compile-time (L, M, T).
// Thread (p, g) owns the R outputs m = m0 + p + g*L*R + r*L, r < R.  They share
// one polyphase branch phi, and their input windows are shifted by M samples,
// so one tap read feeds R FMAs and one window read feeds up to T FMAs:
// (T + (R-1)M) + T LDS reads per R*T FMAs.
//
// For even M every window of a thread starts at the same x parity a, and the
// sum runs two taps per v_pk_fma_f32: the halves of one register pair keep the
// partial sums over the even- and odd-indexed x samples, pair p covering
// x[E + 2p], x[E + 2p + 1] from the even start E = Q - a (Q = q - (T-1), the
// window start) against taps (h[2p - a], h[2p + 1 - a]), h[u] = P[phi][T-1-u]
// (0 outside [0, T)); y = even + odd.  This is the canonical summation order
// of the SRC for even M; the single-pass chain kernel (chain_tile.hip) uses
// it too, so both produce bitwise the same y.  Odd M sums even and odd u in
// two chains (the same partial sums: y = chain 0 + chain 1).
// ---------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int L, int M, int T, int R, int NT>
__global__ __launch_bounds__(NT) void k_src_reg(
    const float* __restrict__ x, float* __restrict__ y, int64_t n_in,
    int64_t ld_x, int64_t n_out, int64_t ld_y, const float* __restrict__ taps,
    int K, int64_t c, int vec_x, int vec_y) {
  constexpr bool PACK = M % 2 == 0;
  constexpr int G = NT / L;          // thread groups with one thread per phase
  constexpr int TILE = G * L * R;    // outputs per block
  constexpr int NP = T / 2 + 1;                           // tap pairs (packed)
  constexpr int TP = PACK ? ((2 * NP + 3) / 4) * 4 : ((T + 3) / 4) * 4 + 4;  // bank row
  constexpr int NROW = PACK ? 2 * L : L;                  // rows: (phi, a) or phi
  constexpr int WMAX = ((TILE - 1) * M) / L + T + 2 + 8;  // window + align slack
  constexpr int WF = ((WMAX + 3) / 4) * 4;
  static_assert(TILE % 4 == 0, "tile must be float4 aligned");

  __shared__ __attribute__((aligned(16))) float s_bank[NROW * TP];
  __shared__ __attribute__((aligned(16))) float s_win[WF];
  __shared__ __attribute__((aligned(16))) float s_out[TILE];
  __shared__ float s_red[NT / 64];

  const int tid = threadIdx.x;
  const int64_t b = blockIdx.y;
  const int64_t m0 = (int64_t)blockIdx.x * TILE;
  const float* xr = x + b * ld_x;
  float* yr = y + b * ld_y;

  const int64_t qlo = (m0 * M + c) / L - (T - 1);
  const int64_t qhi = ((m0 + TILE - 1) * M + c) / L;
  const int64_t qa = qlo & ~(int64_t)3;
  // Packed pairs reach up to 2 samples past the last window (zero taps there).
  const bool nf = load_window<NT>(s_win, xr, qa, (int)(qhi - qa + 1 + (PACK ? 2 : 0)), n_in,
                                  vec_x != 0);
  const float thr = block_flush_threshold<NT>(taps, K, L, s_red);

  // Bank row phi holds the branch taps reversed, h[u] = P[phi][T-1-u]; the
  // packed bank has one row per (phi, a): row[k] = h[k - a].
  for (int i = tid; i < NROW * TP; i += NT) {
    const int row = i / TP, k = i - row * TP;
    const int phi = PACK ? row >> 1 : row, u = PACK ? k - (row & 1) : k;
    const int kk = phi + L * (T - 1 - u);
    s_bank[i] = (u >= 0 && u < T && kk < K) ? flush_tap(taps[kk], thr) : 0.f;
  }
  const bool any_nf = __syncthreads_or(nf);

  if (tid < G * L) {
    const int p = tid % L, g = tid / L;
    const int lbase = p + g * L * R;                 // local index of r = 0
    const int64_t j = (m0 + lbase) * M + c;
    const int64_t q = j / L;
    const int phi = (int)(j - q * L);
    if constexpr (PACK) {
      const int64_t Q = q - (T - 1);
      const int a = (int)(Q & 1);
      const f32x2* w = reinterpret_cast<const f32x2*>(s_win + (int)(Q - a - qa));
      const f32x2* h = reinterpret_cast<const f32x2*>(s_bank + (2 * phi + a) * TP);
      f32x2 acc[R];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = f32x2{0.f, 0.f};
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        const f32x2 t = h[u];
#pragma unroll
        for (int r = 0; r < R; ++r)
          acc[r] = __builtin_elementwise_fma(t, w[r * (M / 2) + u], acc[r]);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) s_out[lbase + r * L] = acc[r].x + acc[r].y;
    } else {
      // odd M: two chains, over even and odd u (round 6: the canonical order,
      // as k_src_generic and the per-phase single-pass kernels sum, so y is
      // bitwise theirs; one chain before)
      const float* w = s_win + (int)(q - (T - 1) - qa);
      const float* h = s_bank + phi * TP;
      float acc[R], acc1[R];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = acc1[r] = 0.f;
#pragma unroll
      for (int u = 0; u < T; ++u) {
        const float t = h[u];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (u & 1) acc1[r] = fmaf(t, w[r * M + u], acc1[r]);
          else acc[r] = fmaf(t, w[r * M + u], acc[r]);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) s_out[lbase + r * L] = acc[r] + acc1[r];
    }
  }
  __syncthreads();
  if (any_nf) {
    // An inf or NaN in the block's window (rare): every output through
    // window_sums / nf_fix (common.h) with the caller's taps.
    for (int i = tid; i < TILE; i += NT) {
      const int64_t j = (m0 + i) * M + c, q = j / L;
      const int base = (int)(q - qa);
      float nfs, fin, v = s_out[i];
      window_sums(taps, K, L, (int)(j - q * L), thr, PACK ? (int)(q & 1) : T - 1,
                  [&](int t) { return s_win[base - t]; }, nfs, fin);
      nf_fix(v, nfs, fin);
      s_out[i] = v;
    }
    __syncthreads();
  }

  const int64_t count = min((int64_t)TILE, n_out - m0);
  store_tile<NT>(yr + m0, s_out, (int)count, vec_y != 0);
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
  __shared__ float s_red[kGenNT / 64];
  const bool nf = load_window<kGenNT>(s_win, xr, qa, (int)(qhi - qa + 1), n_in, vec_x != 0);
  const float thr = block_flush_threshold<kGenNT>(taps, K, L, s_red);
  for (int i = tid; i < L * T; i += kGenNT) {
    const int phi = i / T, u = i - phi * T;
    const int k = phi + L * (T - 1 - u);
    s_bank[i] = (k < K) ? flush_tap(taps[k], thr) : 0.f;
  }
  const bool any_nf = __syncthreads_or(nf);

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
    float v = a0 + a1;
    if (any_nf) {  // an inf or NaN in the block's window (rare): window_sums / nf_fix
      const int base = (int)(q - qa);
      float nfs, fin;
      window_sums(taps, K, L, phi, thr, T - 1, [&](int t) { return s_win[base - t]; }, nfs, fin);
      nf_fix(v, nfs, fin);
    }
    yr[m] = v;
    q += dq;
    phi += dphi;
    if (phi >= L) {
      phi -= L;
      ++q;
    }
  }
}

template <int L, int M, int T, int R, int NT>
int run_reg(const float* x, float* y, int64_t B, int64_t n_in, int64_t ld_x,
            int64_t n_out, int64_t ld_y, const float* taps, int K, int64_t c,
            int vec_x, int vec_y, hipStream_t s) {
  constexpr int TILE = (NT / L) * L * R;
  dim3 grid((unsigned)ceil_div(n_out, TILE), (unsigned)B);
  TraceScope trace("src_poly", s);
  hipLaunchKernelGGL((k_src_reg<L, M, T, R, NT>), grid, dim3(NT), 0, s, x, y,
                     n_in, ld_x, n_out, ld_y, taps, K, c, vec_x, vec_y);
  DSP_LAUNCHED("k_src_reg");
  return DSP_OK;
}

// One launch over B <= kMaxGridY rows (the grid's y extent is the batch).
int launch_src_rows(const float* x, float* y, int64_t B, int64_t n_in, int64_t ld_x,
                    int64_t n_out, int64_t ld_y, const float* taps, int K, int L, int M,
                    int64_t c, hipStream_t s) {
  const int T = (K + L - 1) / L;
  const int vec_x = ((ld_x & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0);
  const int vec_y = ((ld_y & 3) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0);

  // Register-blocked instantiations: the benchmark configurations and the
  // app's most common (L, M) pairs with the default tap rule 40*max(L,M)+1.
  // R is chosen so that R*M is not a multiple of 32: thread groups' windows
  // start R*M floats apart and must land on different LDS banks.
  if (L == 3 && M == 2 && T == 41)
    return run_reg<3, 2, 41, 15, 192>(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, c, vec_x, vec_y,
                                      s);
  if (L == 3 && M == 2 && T == 85)
    return run_reg<3, 2, 85, 7, 192>(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, c, vec_x, vec_y,
                                     s);
  if (L == 2 && M == 1 && T == 64)
    return run_reg<2, 1, 64, 15, 256>(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, c, vec_x, vec_y,
                                      s);
  if (L == 2 && M == 1 && T == 41)
    return run_reg<2, 1, 41, 15, 256>(x, y, B, n_in, ld_x, n_out, ld_y, taps, K, c, vec_x, vec_y,
                                      s);

  // Generic path.  Shrink the tile until bank + window fit in LDS.
  const int bank_floats = ((L * T + 3) / 4) * 4;
  int tile = kGenTile;
  auto lds_bytes = [&](int t) {
    const int64_t w = ((int64_t)(t - 1) * M) / L + T + 2 + 8;
    return (int64_t)(bank_floats + ((w + 3) / 4) * 4) * 4;
  };
  constexpr int64_t kLdsMax = 160 * 1024 - 64;  // (the kernel's static LDS: s_red)
  while (tile > 64 && lds_bytes(tile) > kLdsMax) tile >>= 1;
  if (lds_bytes(tile) > kLdsMax)
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

constexpr int64_t kMaxGridY = 65535;

}  // namespace

int launch_src(const float* x, float* y, int64_t B, int64_t n_in, int64_t ld_x,
               int64_t n_out, int64_t ld_y, const float* taps, int K, int L,
               int M, int64_t c, hipStream_t s) {
  DSP_REQUIRE(B >= 0 && n_in >= 1 && n_out >= 0, "bad sizes B=%lld n_in=%lld n_out=%lld",
              (long long)B, (long long)n_in, (long long)n_out);
  DSP_REQUIRE(L >= 1 && M >= 1 && K >= 1, "bad L=%d M=%d K=%d", L, M, K);
  DSP_REQUIRE(c >= 0, "bad c_offset %lld", (long long)c);
  DSP_REQUIRE(ld_x >= n_in && ld_y >= n_out, "leading dimension too small");
  if (B == 0 || n_out == 0) return DSP_OK;
  DSP_REQUIRE(x && y && taps, "null pointer");
  // Batches beyond the grid's y extent run as consecutive row ranges.
  for (int64_t b0 = 0; b0 < B; b0 += kMaxGridY) {
    const int64_t nb = B - b0 < kMaxGridY ? B - b0 : kMaxGridY;
    if (int rc = launch_src_rows(x + b0 * ld_x, y + b0 * ld_y, nb, n_in, ld_x, n_out, ld_y, taps,
                                 K, L, M, c, s))
      return rc;
  }
  return DSP_OK;
}

}  // namespace dsp
