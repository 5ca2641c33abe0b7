// Single-pass SRC -> biquad cascade, the default path of dsp_chain_f32 (gfx950).
//
// Replaces, for a batch of channels, reference app.py:164-167:
//   y = conversion_tasa_muestreo(x, fs, M, L)   modules/dsp_core.py:133-173
//   z = sistema_ecualizador(y, fs', gains)      modules/dsp_core.py:216-254
// in ONE launch that reads x once and writes y and z once: HBM traffic is the
// algorithmic 4*N_in + 8*N_out bytes per channel, against 4*N_in + 4*N_out
// (SRC kernel) + 4*N_in*rows/shift + 8*N_out (two-pass cascade) for the
// two-launch chain.
//
// Decomposition.  A workgroup is ONE wavefront and owns a tile of 64*TSUB
// consecutive outputs of one channel; lane l owns the sub-chunk of TSUB
// outputs l*TSUB .. l*TSUB + TSUB-1 of the tile, TSUB = 32*L/M, i.e. exactly
// 32 new input samples per lane.  Because TSUB*M is a multiple of L, every
// lane (and every tile) sees the same polyphase pattern: output i of a
// sub-chunk reads x[32*l + qi(i) - t] with branch phi(i) (compile-time), so
// the taps are wave-uniform (scalar loads) and each lane runs
//   1. SRC: y[i] = sum_u P[phi(i)][TT-1-u] * w[qi(i) + u] from its 72-sample
//      window, read from the tile's x window in LDS (one coalesced load per
//      tile, padded so the 64 lanes' ds_read_b128 are conflict-free).  Same
//      per-output FMA order as k_src_reg: y is bitwise the SRC kernel's.
//   2. pass 1: the sub-chunk's zero-state end state.  The sums run in float32
//      (v_pk_fma_f32, 6 per sample) in INPUT-NORMAL coordinates xi = P^-1 w
//      (P P^T = the cascade's state covariance under unit white noise, so every
//      coordinate has unit variance and the float32 sums do not cancel):
//      e_l = sum_i Gc[i] y[i], Gc[i] = P^-1 A^(TSUB-1-i) B (wave-uniform);
//      then one float64 change of basis E'_l = Q e_l, Q = T^-1 P (lower
//      triangular, 78 FMAs per lane), into block-diagonal coordinates (below);
//   3. carry: the tile's entry state m_in comes from the previous tile of the
//      same channel (chained hand-off, below); a blocked scan of the 64
//      lanes' E' through LDS (tile_cascade) gives every sub-chunk's entry
//      state m_l = v_(l-1), v_l = D^TSUB v_(l-1) + E'_l, v_(-1) = m_in;
//   4. v_63 (the tile's end state) is published for the next tile;
//   5. y leaves through LDS as coalesced float4 stores; the lane's DF2 state
//      is s_l = T m_l and pass 2 reruns the cascade over the sub-chunk from it,
//      clips, and z leaves the same way.
//
// Block-diagonal coordinates.  The cascade's state matrix A is block lower
// triangular (stage k is driven by stage k-1's output) with 2x2 diagonal
// blocks A_kk.  With T block unit lower triangular solving A T = T D,
// D = diag(A_kk) (Sylvester equations A_ii X - X A_jj = C for the off-diagonal
// blocks, solvable when no two stages share a pole pair), A^N = T D^N T^-1 and
// powers of D are six independent 2x2 powers: the carry costs 4 FMAs per block
// per scan level instead of a dense 12x12 product.  Stages that only pad the
// cascade to six (exact identities) have states no output depends on; their
// coordinates are dropped.  The host computes T, D's powers and checks the
// conditioning in float64; a cascade without a well-conditioned T takes the
// two-launch chain.
// y never returns from HBM, and there is no second pass over x.
//
// Chained hand-off.  Workgroups are numbered tile-major (id = tile*B + b), so
// tile t-1 of a channel was dispatched B workgroups before tile t; at B >= the
// chip's resident wave count its end state is normally published long before
// tile t needs it.  A workgroup waits only on a lower id, and ids are
// dispatched in order, so every wait ends.  The state (12 doubles) and its
// flag are agent-scope atomics (global loads/stores with sc1: coherent at
// device scope across the XCDs' L2s, per location).  The producer lane stores
// the payload, waits vmcnt(0) (every payload store acknowledged) and only then
// stores the flag; the consumer polls the flag and issues the payload loads
// only after a poll returned 1 (a control dependency on a returned value, and
// asm memory clobbers keep the compiler from hoisting them).  Ordering between
// the payload and the flag therefore rests on the gfx950 ISA, not on C++
// release/acquire: the memory model's agent-scope release/acquire fences add
// buffer_wbl2 sc1 / buffer_inv sc1 (L2 write-back / invalidate), which the
// atomics do not need and which measured 5.8x slower (config 4: 37.7 vs
// 6.55 ms, profiles/r03_handoff_fence_ab.txt).  The consumer clears the flag, so a completed launch leaves
// the flag array zero for the next one (the caller zero-fills the workspace
// once).  Round 4: the producer raises its flag once the state stores are
// acknowledged but after its y stores are issued (a counted vmcnt), and
// k_chain_tile's consumer polls once before its x window loads: if the flag
// is already up (the common case: the producer ran a dispatch generation
// earlier), the state comes by an sc1 LDS-DMA issued after that poll, behind
// the SRC and pass 1 (chain_tile_body); else it waits as described.  A wait that polls more than the thread's spin limit
// (dsp_chain_spin_limit; default 2^23 polls with s_sleep 2 between them,
// ~0.4 s: a broken dispatch order, or a GPU time-sliced between processes)
// gives up: it sets the workspace's status word (dsp_chain_status reports it,
// Chain.run raises) and leaves the flag for the workspace reset; z of that
// launch is wrong, nothing hangs.
//
// Rows are bitwise independent of the batch size: the geometry depends on
// (L, M, K) only.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>

#include "cascade.h"

#include "chain_pp.h"
#include "chain_tile.h"

namespace dsp {
namespace {

// One tile of the L3/M2 kernel (REPAIR: the rerun with the non-finite path).
// MODE: 0 the chained hand-off, 1 / 2 launch 1 / 3 of the three-launch mode
// (chain_tile.h, AggEntry / GivenEntry).
template <class GEO, bool DLY, bool REPAIR, int MODE = 0>
__device__ __forceinline__ void chain_tile_body(const TileArgs& a, float* lds, int lane, int64_t b,
                                                int64_t tile) {
  constexpr int TS = GEO::TSUB;
  const int64_t m0 = tile * GEO::TILE;  // first output of the tile
  const tt_ptr mt = (tt_ptr)a.tt;       // wave-uniform: scalar loads

  // Early hand-off (not in the repair rerun): lane 0 polls the previous
  // tile's flag once now, ahead of the x window loads; if it is raised, the
  // state follows by an agent-scope (sc1) LDS-DMA into the slot after the
  // window -- issued after the poll returned, as the hand-off protocol
  // requires -- and arrives behind the SRC and pass 1 instead of two global
  // round trips after them.  Otherwise tile_cascade waits as before.
  uint32_t fl = 0;
  if (!REPAIR && MODE == 0 && tile > 0 && lane == 0)
    fl = load_flag(a.flags + b * a.ntiles + tile - 1);

  // ---- x window of the tile -> padded LDS image (x == 0 outside [0, n_in))
  {
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.x) + b * a.ld_x, 0, (int)(a.n_in * 4), 0x00020000);
    const int64_t xs0 = m0 * GEO::M / GEO::L + a.cq - (GEO::TT - 1);  // multiple of 4
    constexpr int NF = GEO::NWIN / 4;
    // The lane's float4s f = lane + 64 k: buffer byte (xs0 + 4 f) * 4 = off0 +
    // 1024 k and LDS float xpad(4 f) = l0 + 288 k (lane < 64), one address
    // register each with k in the instructions' offsets.
    const int off0 = (int)(xs0 * 4) + 16 * lane;
    float* const l0 = lds + 4 * lane + 4 * (lane >> 3);
#pragma unroll
    for (int k = 0; k < (NF + kWave - 1) / kWave; ++k) {
      if ((k + 1) * kWave <= NF || lane + kWave * k < NF) {
        // "Negative" offsets (tile 0) are >= 2^31 as unsigned: out of range, zeros.
        const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rx, off0 + 1024 * k, 0, kStream);
        *reinterpret_cast<f32x4*>(l0 + 288 * k) = v;
      }
    }
    static_assert(xpad(4 * (kWave + 7)) - xpad(4 * 7) == 288, "xpad: 288 floats per 64 float4s");
  }
  fence();  // one wave: its LDS operations execute in order
  EarlyEntry early{false, reinterpret_cast<const double*>(lds + GEO::LDSF)};
  if (!REPAIR && MODE == 0 && tile > 0 && __builtin_amdgcn_readfirstlane(fl) == 1u) {
    early.early = true;
    if (lane < 2 * kD) {
      const int64_t prev = b * a.ntiles + tile - 1;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(reinterpret_cast<const uint32_t*>(
                                                               a.states + prev * kD) + lane),
          (__attribute__((address_space(3))) void*)(lds + GEO::LDSF), 4, 0, kSc1);
    }
  }

  // ---- 1. SRC: the lane's TSUB outputs, in parts (register pressure)
  float y[TS];
  {
    const float* xw = lds + 36 * lane;
    static_assert(TS == 48, "SRC parts of 48 / 24 outputs");
    // DLY: one part of 48 (its delay outputs need no accumulators: 128 VGPRs,
    // no scratch); the plain kernel in two parts of 24 (one part would spill).
    if constexpr (DLY) {
      src_part<GEO, 0, 48, true>(xw, mt, y);
      pin(y);
    } else {
      src_part<GEO, 0, 24, false>(xw, mt, y);
      pin(y);
      src_part<GEO, 24, 24, false>(xw, mt, y);
      pin(y);
    }
  }
  if constexpr (REPAIR) {
    // each output's reference sums over its window (window_sums, nf_fix)
    auto fix = [&](float (&yy)[TS], double (&v)[kD]) {
      const float thr = mt->flush_thr;
      fix_outputs(a, mt, b, m0 + TS * lane, yy, v, [&](int i, float& nf, float& fin) {
        const int j = i * GEO::M + GEO::CR;
        const int base = kLS * lane + j / GEO::L + GEO::TT - 1;  // window offset of x[q]
        // (window starts and q keep x's absolute parity: xs0 is a multiple of 4)
        window_sums(a.taps, a.K, GEO::L, j % GEO::L, thr, base,
                    [&](int t) { return lds[xpad(base - t)]; }, nf, fin);
      });
    };
    tile_cascade<TS, true, true>(a, mt, lds, y, lane, b, tile, m0, fix);
  } else if constexpr (MODE == 1) {
    tile_cascade<TS>(a, mt, lds, y, lane, b, tile, m0, 0, AggEntry{});
  } else if constexpr (MODE == 2) {
    tile_cascade<TS>(a, mt, lds, y, lane, b, tile, m0, 0, GivenEntry{});
  } else {
    tile_cascade<TS>(a, mt, lds, y, lane, b, tile, m0, 0, early);
  }
}

template <class GEO, bool DLY = false>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(4))) void k_chain_tile(
    TileArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[GEO::LDSF + 2 * kD];  // + the early slot
  // grid (B, ntiles): linear ids tile-major (x fastest), no division
  const int64_t tile = blockIdx.y, b = blockIdx.x;
  chain_tile_body<GEO, DLY, false>(a, lds, threadIdx.x, b, tile);
}

// Launches 1 and 3 of the three-launch mode (chain_tile.h, AggEntry).
template <class GEO, bool DLY, int MODE>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(4))) void k_chain_tile3(
    TileArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[GEO::LDSF];
  chain_tile_body<GEO, DLY, false, MODE>(a, lds, threadIdx.x, blockIdx.x, blockIdx.y);
}

template <class GEO, bool DLY = false>
__global__ __launch_bounds__(kWave) void k_chain_tile_repair(TileArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[GEO::LDSF + 2 * kD];  // + the early slot
  repair_channels(a, 0, 1, [&](int64_t b, int64_t tile) {
    chain_tile_body<GEO, DLY, true>(a, lds, (int)threadIdx.x, b, tile);
  });
}

// ---------------------------------------------------------------------------
// Generic single-pass kernel: any L, M with ceil(K/L) <= 8 (config 5's
// L/M = 160/147, K = 1023: 7 taps per branch) and at most 8 phase classes.
// The polyphase branch of a lane's outputs changes from output to output and
// from lane to lane:
//   j = m*M + c, phi = j mod L, q = j div L,
//   y[m] = sum_u h[phi][u] x[q - (T-1) + u],  h[phi][u] = taps[phi + L(T-1-u)],
// summed as k_src_generic does (even u and odd u in two chains, y = even +
// odd), so y is bitwise that kernel's.  Sub-chunks start at outputs m = 32 j,
// and their branch sequences repeat with j mod C, C = L / gcd(32 M mod L, L)
// (5 for 160/147): the host tabulates every class's 32 rows of taps and its
// q-advance bits (TileTables::seq/adv), so a lane's taps for output i sit at a
// compile-time offset of its class row and the SRC does no phase arithmetic.
// A workgroup is kGenWaves waves, one channel each at the same tile index
// (ids stay tile-major for the hand-off); they share the class tables in LDS.
// Each wave owns its x window (and stages its stores through it).  Steps 2-5
// are tile_cascade<32>.
// ---------------------------------------------------------------------------
// The generic kernels' workgroup: kGenWaves waves, wave w takes channel
// g kGenWaves + w of channel group g; the ids are tile-major over groups.
__device__ __forceinline__ int gen_wave() {
  return __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
}

// Tile x window of a generic kernel's wave: x[qa .. qa + a.win) (zeros
// outside [0, n_in)), 8 float4 loads in flight per lane per round.
__device__ __forceinline__ void gen_load_window(const TileArgs& a, float* win, int lane, int64_t b,
                                                int64_t qa) {
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.x) + b * a.ld_x, 0, (int)(a.n_in * 4), 0x00020000);
  const int nf = a.win >> 2;
  for (int f0 = 0; f0 < nf; f0 += 8 * kWave) {
    f32x4 v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int f = f0 + r * kWave + lane;  // past the window: harmless reads
      v[r] = __builtin_amdgcn_raw_buffer_load_b128(rx, (int)((qa + 4 * f) * 4), 0, kStream);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int f = f0 + r * kWave + lane;
      if (f < nf) *reinterpret_cast<f32x4*>(win + 4 * f) = v[r];
    }
  }
}

// Class tables of k_chain_gen into LDS (class stride kGenClassStride floats:
// the rows that lanes of different classes read together start on distinct
// bank quads), then the advance masks; two float4 loads in flight per thread.
// Ends with a workgroup barrier.
__device__ __forceinline__ void gen_load_classes(const TileArgs& a, float* seq, uint32_t* adv) {
  constexpr int kNT = kWave * kGenWaves;
  constexpr int kF4 = kGenTS * kGenTT / 4;  // float4s per class
  const int C = ((tt_ptr)a.tt)->classes;
  const f32x4* src = reinterpret_cast<const f32x4*>(a.tt->seq);
  f32x4 v[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) v[r] = src[(r * kNT + threadIdx.x) & (kGenClasses * kF4 - 1)];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int i = r * kNT + threadIdx.x, k = i / kF4, f = i - k * kF4;
    if (k < C) *reinterpret_cast<f32x4*>(seq + k * kGenClassStride + 4 * f) = v[r];
  }
  if (threadIdx.x < kGenClasses) adv[threadIdx.x] = a.tt->adv[threadIdx.x];
  __syncthreads();
}

// The generic kernels' on_nf for the repair rerun: window x[qa ..] unpadded
// in `win`, the lane's outputs m0 + 32 lane + i with j0 = (m0 + 32 lane) M + c.
__device__ __forceinline__ void gen_fix(const TileArgs& a, tt_ptr mt, const float* win, int64_t qa,
                                        int64_t j0, int64_t b, int64_t z0, float (&yy)[kGenTS],
                                        double (&v)[kD]) {
  const float thr = mt->flush_thr;
  fix_outputs(a, mt, b, z0, yy, v, [&](int i, float& nf, float& fin) {
    const int64_t j = j0 + (int64_t)i * a.M, q = j / a.L;
    const int base = (int)(q - qa);
    window_sums(a.taps, a.K, a.L, (int)(j - q * a.L), thr, a.T - 1,
                [&](int t) { return win[base - t]; }, nf, fin);
  });
}

// One tile of k_chain_gen for one wave (REPAIR: the rerun with the
// non-finite path).
template <bool UP, bool REPAIR, class ENTRY = ChainedEntry>
__device__ __forceinline__ void chain_gen_body(const TileArgs& a, const float* seq,
                                               const uint32_t* adv, float* win, int lane,
                                               int64_t b, int64_t tile, ENTRY&& entry = ENTRY{}) {
  const int L = a.L, M = a.M, T = a.T;
  const tt_ptr mt = (tt_ptr)a.tt;
  const int C = mt->classes;
  const int64_t m0 = tile * kGenTile;

  // ---- x window of the tile
  const int64_t qlo = (m0 * M + a.c) / L - (T - 1);
  const int64_t qa = (qlo >> 2) << 2;  // floor to a multiple of 4
  gen_load_window(a, win, lane, b, qa);
  fence();

  // ---- 1. SRC of the lane's 32 outputs, software-pipelined one output deep
  // (output i+1's LDS reads are issued before output i's FMAs).  UP (M < L):
  // q advances by 0 or 1 per output, so the 8-sample window slides in
  // registers and one new sample is read per output; otherwise all 8 are read.
  // (j = m M + c in 32 bits: tile_geometry keeps n_out M + c below 2^31)
  float y[kGenTS];
  const int64_t j0 = (m0 + (int64_t)kGenTS * lane) * M + a.c;
  {
    const int jl = (int)(m0 * M + a.c) + kGenTS * M * lane;
    int qr = jl / L - (T - 1) - (int)qa;  // window offset of the output's first tap
    const int dq = M / L;
    const int cls = ((int)tile * kWave + lane) % C;  // sub-chunk j = m0/32 + lane
    const float* row = seq + cls * kGenClassStride;   // output i's taps at row + 8 i
    const uint32_t am = adv[cls];
    float w[kGenTT];
#pragma unroll
    for (int u = 0; u < kGenTT; ++u) w[u] = win[qr + u];
    float4 h0 = *reinterpret_cast<const float4*>(row);
    float4 h1 = *reinterpret_cast<const float4*>(row + 4);
    float nx = UP ? win[qr + kGenTT] : 0.f;  // enters the window if q advances
#pragma unroll
    for (int i = 0; i < kGenTS; ++i) {
      // operands of output i+1
      const bool carry = (am >> i) & 1u;
      const int qr_n = qr + dq + (carry ? 1 : 0);
      float4 h0n, h1n;
      float nxn = 0.f, wn[kGenTT];
      if (i + 1 < kGenTS) {
        h0n = *reinterpret_cast<const float4*>(row + kGenTT * (i + 1));
        h1n = *reinterpret_cast<const float4*>(row + kGenTT * (i + 1) + 4);
        if constexpr (UP) {
          nxn = win[qr_n + kGenTT];
        } else {
#pragma unroll
          for (int u = 0; u < kGenTT; ++u) wn[u] = win[qr_n + u];
        }
      }
      // (even u, odd u) partial sums in the halves of one v_pk_fma_f32
      // chain: the same two chains, in the same order, as k_src_generic's.
      f32x2 acc = {0.f, 0.f};
      acc = __builtin_elementwise_fma(f32x2{h0.x, h0.y}, f32x2{w[0], w[1]}, acc);
      acc = __builtin_elementwise_fma(f32x2{h0.z, h0.w}, f32x2{w[2], w[3]}, acc);
      acc = __builtin_elementwise_fma(f32x2{h1.x, h1.y}, f32x2{w[4], w[5]}, acc);
      acc = __builtin_elementwise_fma(f32x2{h1.z, h1.w}, f32x2{w[6], w[7]}, acc);
      y[i] = acc.x + acc.y;
      if (i + 1 < kGenTS) {
        if constexpr (UP) {
#pragma unroll
          for (int u = 0; u < kGenTT - 1; ++u) w[u] = carry ? w[u + 1] : w[u];
          w[kGenTT - 1] = carry ? nx : w[kGenTT - 1];
          nx = nxn;
        } else {
#pragma unroll
          for (int u = 0; u < kGenTT; ++u) w[u] = wn[u];
        }
        h0 = h0n;
        h1 = h1n;
        qr = qr_n;
      }
    }
  }
  pin(y);
  if constexpr (REPAIR)
    tile_cascade<kGenTS, true, true>(a, mt, win, y, lane, b, tile, m0,
                                     [&](float (&yy)[kGenTS], double (&v)[kD]) {
                                       gen_fix(a, mt, win, qa, j0, b, m0 + kGenTS * lane, yy, v);
                                     });
  else
    tile_cascade<kGenTS>(a, mt, win, y, lane, b, tile, m0, 0, entry);
}

template <bool UP>
__global__ __launch_bounds__(kWave * kGenWaves) __attribute__((amdgpu_waves_per_eu(4))) void
k_chain_gen(TileArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int w = gen_wave();
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t tile = blockIdx.y;  // grid (groups, ntiles): tile-major
  const int64_t b = (int64_t)blockIdx.x * kGenWaves + w;
  float* seq = smem;
  uint32_t* adv = reinterpret_cast<uint32_t*>(smem + kGenClasses * kGenClassStride);
  gen_load_classes(a, seq, adv);
  if (b >= a.B) return;
  float* win = smem + kGenClasses * kGenClassStride + kGenClasses + w * a.win;
  chain_gen_body<UP, false>(a, seq, adv, win, lane, b, tile);
}

// Launches 1 and 3 of the three-launch mode (chain_tile.h, AggEntry).
template <bool UP, int MODE>
__global__ __launch_bounds__(kWave * kGenWaves) __attribute__((amdgpu_waves_per_eu(4))) void
k_chain_gen3(TileArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int w = gen_wave();
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t tile = blockIdx.y;
  const int64_t b = (int64_t)blockIdx.x * kGenWaves + w;
  float* seq = smem;
  uint32_t* adv = reinterpret_cast<uint32_t*>(smem + kGenClasses * kGenClassStride);
  gen_load_classes(a, seq, adv);
  if (b >= a.B) return;
  float* win = smem + kGenClasses * kGenClassStride + kGenClasses + w * a.win;
  if constexpr (MODE == 1) chain_gen_body<UP, false>(a, seq, adv, win, lane, b, tile, AggEntry{});
  else chain_gen_body<UP, false>(a, seq, adv, win, lane, b, tile, GivenEntry{});
}

template <bool UP>
__global__ __launch_bounds__(kWave * kGenWaves) void k_chain_gen_repair(TileArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int w = gen_wave();
  const int lane = threadIdx.x & (kWave - 1);
  float* seq = smem;
  uint32_t* adv = reinterpret_cast<uint32_t*>(smem + kGenClasses * kGenClassStride);
  gen_load_classes(a, seq, adv);
  float* win = smem + kGenClasses * kGenClassStride + kGenClasses + w * a.win;
  repair_channels(a, w, kGenWaves, [&](int64_t b, int64_t tile) {
    chain_gen_body<UP, true>(a, seq, adv, win, lane, b, tile);
  });
}

// ---------------------------------------------------------------------------
// Select-free generic kernel for a compile-time ratio M < L (config 5's
// 160/147).  Output i of a lane reads x[q_i - (T-1) + u], q_i = q_0 + g_i +
// d_i with g_i = i M div L (compile-time) and d_i in {0, 1} (the class's
// phase carry).  The host folds d_i and the parity of g_i into the class rows
// (TileTables::seqs: T taps shifted by 0..2 in 10 slots), so output i sums
// its row against the window pairs from g_i rounded down to even -- registers
// at compile-time indices: no window sliding, no per-lane selects.  A shift
// of 1 swaps which half of the v_pk_fma_f32 holds the even-u and the odd-u
// chain; the extra slots hold zero taps (x * 0 + acc == acc, and +0 stays
// +0), so y = even + odd is bitwise k_chain_gen's and k_src_generic's.
// ---------------------------------------------------------------------------
// T7 (T <= 7 taps per branch, config 5's K = 1023): an output whose g_i is
// even has shift d_i in {0, 1}, so its taps fill slots 0..7 and slots 8, 9 are
// zero: the last tap-pair read and FMA are skipped (bitwise the same y).
constexpr int ct_gcd(int a, int b) { return b ? ct_gcd(b, a % b) : a; }

// Class rows of k_chain_gct into LDS (the C classes in use only).  Ends with
// a workgroup barrier.
__device__ __forceinline__ void ct_load_classes(const TileArgs& a, float* seq) {
  constexpr int kF4 = kGenTS * kCtRow / 4;  // float4s per class
  const int C = ((tt_ptr)a.tt)->classes;
  const f32x4* src = reinterpret_cast<const f32x4*>(&a.tt->seqs[0][0][0]);
  for (int i = threadIdx.x; i < C * kF4; i += kWave * kGenWaves) {
    const int k = i / kF4, f = i - k * kF4;
    *reinterpret_cast<f32x4*>(seq + k * kCtClassStride + 4 * f) = src[i];
  }
  __syncthreads();
}

// x offset (a multiple of 4) of the x window of a generic kernel's tile.
template <int L, int M>
__device__ __forceinline__ int64_t gen_window_start(const TileArgs& a, int64_t tile) {
  const int64_t qlo = (tile * kGenTile * M + a.c) / L - (a.T - 1);
  return (qlo >> 2) << 2;
}

// Steps 1-5 of one tile of k_chain_gct for one wave whose x window x[qa ..]
// is in `win` (REPAIR: the rerun with the non-finite path; entry:
// tile_cascade's).
template <int L, int M, bool T7, bool REPAIR, int G = 2, class ENTRY = ChainedEntry>
__device__ __forceinline__ void gct_tile(const TileArgs& a, const float* seq, float* win,
                                         int lane, int64_t b, int64_t tile, int64_t qa,
                                         ENTRY&& entry = ENTRY{}) {
  static_assert(M < L, "q advances by 0 or 1 per output");
  constexpr int NPW = ((kGenTS - 1) * M / L) / 2 + kCtTaps / 2;  // window pairs per lane
  const int T = a.T;
  // (opaque: in the persistent kernel's tile loop, table loads stay where
  // they are used instead of hoisted out of the loop into live registers)
  tt_ptr mt = (tt_ptr)a.tt;
  asm volatile("" : "+s"(mt));
  // the phase classes of the 32-output sub-chunk starts, known at compile
  // time for the ratio (gen_classes; the host checked the tables hold as many)
  constexpr int C = L / ct_gcd((kGenTS * M) % L, L);
  const int64_t m0 = tile * kGenTile;

  // ---- 1. SRC of the lane's 32 outputs from its register window
  // (j = m M + c in 32 bits: tile_geometry keeps n_out M + c below 2^31)
  float y[kGenTS];
  const int64_t j0 = (m0 + (int64_t)kGenTS * lane) * M + a.c;
  {
    const int jl = (int)(m0 * M + a.c) + kGenTS * M * lane;
    const float* xl = win + (jl / L - (T - 1) - (int)qa);
    const float* row = seq + (((int)tile * kWave + lane) % C) * kCtClassStride;
    f32x2 X[NPW];
#pragma unroll
    for (int m = 0; m < NPW; ++m) X[m] = f32x2{xl[2 * m], xl[2 * m + 1]};
    // Outputs in groups of G, the next group's tap rows read while this one
    // computes and the G FMA chains interleaved (each output's own chain,
    // groups in ascending order, is unchanged: y bitwise the same).  G = 2
    // against one output at a time: 1.128 -> 1.122 ms at config 5
    // (profiles/r04_gct_pairs_ab.txt); groups of 4 spill at 4 waves per SIMD
    // and pay at the persistent kernel's 3 (profiles/r05_gcp_ab.txt).
    static_assert(kGenTS % G == 0, "whole groups");
    struct Row {
      f32x4 t0, t1;
      f32x2 t2;
    };
    auto load_row = [&](int i) {
      Row r;
      r.t0 = *reinterpret_cast<const f32x4*>(row + kCtRow * i);
      r.t1 = *reinterpret_cast<const f32x4*>(row + kCtRow * i + 4);
      if (!(T7 && ((i * M / L) % 2 == 0)))
        r.t2 = *reinterpret_cast<const f32x2*>(row + kCtRow * i + 8);
      else
        r.t2 = f32x2{0.f, 0.f};
      return r;
    };
    Row cur[G];
#pragma unroll
    for (int o = 0; o < G; ++o) cur[o] = load_row(o);
#pragma unroll
    for (int i0 = 0; i0 < kGenTS; i0 += G) {
      Row nxt[G];
      if (i0 + G < kGenTS) {
#pragma unroll
        for (int o = 0; o < G; ++o) nxt[o] = load_row(i0 + G + o);
      }
      f32x2 acc[G];
#pragma unroll
      for (int o = 0; o < G; ++o) acc[o] = f32x2{0.f, 0.f};
#pragma unroll
      for (int pp = 0; pp < 5; ++pp) {
#pragma unroll
        for (int o = 0; o < G; ++o) {
          const int i = i0 + o;
          const int g2 = (i * M / L) / 2;
          const bool last = !(T7 && ((i * M / L) % 2 == 0));
          if (pp == 4 && !last) continue;
          const f32x2 t = pp == 0   ? f32x2{cur[o].t0.x, cur[o].t0.y}
                          : pp == 1 ? f32x2{cur[o].t0.z, cur[o].t0.w}
                          : pp == 2 ? f32x2{cur[o].t1.x, cur[o].t1.y}
                          : pp == 3 ? f32x2{cur[o].t1.z, cur[o].t1.w}
                                    : cur[o].t2;
          acc[o] = __builtin_elementwise_fma(t, X[g2 + pp], acc[o]);
        }
      }
#pragma unroll
      for (int o = 0; o < G; ++o) y[i0 + o] = acc[o].x + acc[o].y;
#pragma unroll
      for (int o = 0; o < G; ++o) cur[o] = nxt[o];
    }
  }
  pin(y);
  if constexpr (REPAIR)
    tile_cascade<kGenTS, true, true>(a, mt, win, y, lane, b, tile, m0,
                                     [&](float (&yy)[kGenTS], double (&v)[kD]) {
                                       gen_fix(a, mt, win, qa, j0, b, m0 + kGenTS * lane, yy, v);
                                     });
  else
    tile_cascade<kGenTS>(a, mt, win, y, lane, b, tile, m0, 0, entry);
}

// One tile of k_chain_gct for one wave: its x window, then gct_tile.
template <int L, int M, bool T7, bool REPAIR, class ENTRY = ChainedEntry>
__device__ __forceinline__ void chain_gct_body(const TileArgs& a, const float* seq, float* win,
                                               int lane, int64_t b, int64_t tile,
                                               ENTRY&& entry = ENTRY{}) {
  const int64_t qa = gen_window_start<L, M>(a, tile);
  gen_load_window(a, win, lane, b, qa);
  fence();
  gct_tile<L, M, T7, REPAIR>(a, seq, win, lane, b, tile, qa, entry);
}

template <int L, int M, bool T7 = false>
__global__ __launch_bounds__(kWave * kGenWaves) __attribute__((amdgpu_waves_per_eu(4))) void
k_chain_gct(TileArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int w = gen_wave();
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t tile = blockIdx.y;  // grid (groups, ntiles): tile-major
  const int64_t b = (int64_t)blockIdx.x * kGenWaves + w;
  float* seq = smem;
  ct_load_classes(a, seq);
  if (b >= a.B) return;
  float* win = smem + ((tt_ptr)a.tt)->classes * kCtClassStride + w * a.win;
  chain_gct_body<L, M, T7, false>(a, seq, win, lane, b, tile);
}

// Launches 1 and 3 of the three-launch mode (chain_tile.h, AggEntry).
template <int L, int M, bool T7, int MODE>
__global__ __launch_bounds__(kWave * kGenWaves) __attribute__((amdgpu_waves_per_eu(4))) void
k_chain_gct3(TileArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int w = gen_wave();
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t tile = blockIdx.y;
  const int64_t b = (int64_t)blockIdx.x * kGenWaves + w;
  float* seq = smem;
  ct_load_classes(a, seq);
  if (b >= a.B) return;
  float* win = smem + ((tt_ptr)a.tt)->classes * kCtClassStride + w * a.win;
  if constexpr (MODE == 1) chain_gct_body<L, M, T7, false>(a, seq, win, lane, b, tile, AggEntry{});
  else chain_gct_body<L, M, T7, false>(a, seq, win, lane, b, tile, GivenEntry{});
}

template <int L, int M, bool T7 = false>
__global__ __launch_bounds__(kWave * kGenWaves) void k_chain_gct_repair(TileArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int w = gen_wave();
  const int lane = threadIdx.x & (kWave - 1);
  float* seq = smem;
  ct_load_classes(a, seq);
  float* win = smem + ((tt_ptr)a.tt)->classes * kCtClassStride + w * a.win;
  repair_channels(a, w, kGenWaves, [&](int64_t b, int64_t tile) {
    chain_gct_body<L, M, T7, true>(a, seq, win, lane, b, tile);
  });
}

// Persistent k_chain_gct (round 4), for batches of at least a chip's worth of
// workgroups: a workgroup loads the class rows once and walks channel groups
// (grid-stride); each wave runs its channel's tiles in order, carrying the
// end state in registers (RegCarry: no hand-off, no flags, no tile waiting on
// another workgroup).  Every tile's end state is still published for the
// repair kernel.  Rows are bitwise the chained kernel's: the same tile code on
// the same entry states.  Config 5 (8192 channels): 1.134-1.137 vs
// 1.191-1.200 ms same box (profiles/r04_gcp_ab.txt).
// Round 5: 3 waves per SIMD (up to 168 VGPRs) instead of 4, which buys (a) the
// next tile's x window in flight in registers behind the whole current tile
// -- loaded as soon as this tile's window is in LDS, the next channel's tile 0
// behind a channel's last tile -- and (b) the SRC in groups of 4 outputs:
// 1.116 -> 1.094 ms same box (profiles/r05_gcp_ab.txt; (a) alone 1.098).  At 4
// waves per SIMD half the window in flight measured the same and the whole
// window spilled (round 4); an LDS-DMA into a second window slot does not fit
// the LDS, and stores straight from registers instead of store_tile's LDS
// staging, which would free the slot, ran 1.6x (default cache policy) to 6x
// (nt) slower (16-byte pieces 128 bytes apart).
constexpr int kGcpWin = 8;  // float4 per lane of a tile's x window (a.win <= 4 * 8 * 64)

template <int L, int M, bool T7 = false>
__global__ __launch_bounds__(kWave * kGenWaves) __attribute__((amdgpu_waves_per_eu(3))) void
k_chain_gcp(TileArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int w = gen_wave();
  const int64_t groups = (a.B + kGenWaves - 1) / kGenWaves;
  float* seq = smem;
  ct_load_classes(a, seq);
  float* win = smem + ((tt_ptr)a.tt)->classes * kCtClassStride + w * a.win;
  const int nf = a.win >> 2;
  f32x4 v[kGcpWin];
  auto load = [&](int64_t bb, int64_t tile) {
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.x) + bb * a.ld_x, 0, (int)(a.n_in * 4), 0x00020000);
    const int64_t qa = gen_window_start<L, M>(a, tile);
    const int ln = lane_id();
#pragma unroll
    for (int r = 0; r < kGcpWin; ++r)  // past the window: harmless reads
      v[r] = __builtin_amdgcn_raw_buffer_load_b128(rx, (int)((qa + 4 * (r * kWave + ln)) * 4), 0,
                                                   kStream);
  };
  if ((int64_t)blockIdx.x * kGenWaves + w < a.B) load((int64_t)blockIdx.x * kGenWaves + w, 0);
  for (int64_t g = blockIdx.x; g < groups; g += gridDim.x) {
    const int64_t b = g * kGenWaves + w;
    if (b >= a.B) break;  // the last group's missing channels (wave-uniform)
    RegCarry carry{0.0, 0.0};
    for (int64_t tile = 0; tile < a.ntiles; ++tile) {
      const int64_t qa = gen_window_start<L, M>(a, tile);
      {
        const int ln = lane_id();
#pragma unroll
        for (int r = 0; r < kGcpWin; ++r) {
          // (rows r < kGcpWin - 1 are whole: the launcher checks nf; one exec
          // mask instead of eight)
          const int f = r * kWave + ln;
          if (r < kGcpWin - 1 || f < nf) *reinterpret_cast<f32x4*>(win + 4 * f) = v[r];
        }
      }
      fence();
      if (tile + 1 < a.ntiles) {
        load(b, tile + 1);
      } else {
        const int64_t bn = b + (int64_t)gridDim.x * kGenWaves;
        if (bn < a.B) load(bn, 0);
      }
      // (an opaque lane per tile: what the tile derives from it is recomputed
      // instead of hoisted out of the loop and held through it)
      int ln = lane_id();
      asm volatile("" : "+v"(ln));
      gct_tile<L, M, T7, false, 4>(a, seq, win, ln, b, tile, qa, carry);
    }
  }
}

// Instantiated geometries: (L, M, ceil(K/L), c mod L).  (3, 2, 41, 0) is the
// benchmark's L3/M2 with the default K = 121 (configs 3 and 4).
typedef TileGeo<3, 2, 41, 0> Geo3241;

struct TilePlan {
  int kind;  // 1: k_chain_tile<Geo3241>, 2: k_chain_gen, 3: k_chain_gct<160, 147>,
             // 4: k_chain_pp<PpGeo<...>> (chain_pp.h)
  int64_t tsub, tile, ntiles;
  int win;   // kind 2: floats of a wave's x window
  int pp;    // kind 4: the entry of chain_pp_list.h
};

// The per-phase kernels' instantiations (chain_pp_list.h, tools/gen_chain_pp.py).
constexpr PpEntry kPpEntries[] = {
#define PP_GEO(IDX, LR, MR, TS, NP, UC, NH, PB) {LR, MR, TS, NP, UC, NH, PB},
#include PP_LIST
#undef PP_GEO
};
constexpr int kPpCount = (int)(sizeof(kPpEntries) / sizeof(kPpEntries[0]));

// What a call's geometry needs of a per-phase kernel (chain_pp.h, file
// comment): the reduced ratio, the window alignment A and the first window
// sample xa0 of tile 0, r0 and rho, the slot count P, the tap pairs NP of the
// widest slot row and the delay branch's centre offset UC (-1: no delay
// branch, downsampling).
struct PpNeed {
  int g, LR, MR, T, A, r0, rho, P, npmin, UC;
  int64_t xa0;
};

int64_t floor_mod(int64_t a, int64_t m) { return ((a % m) + m) % m; }
int64_t floor_div(int64_t a, int64_t m) { return (a - floor_mod(a, m)) / m; }

PpNeed pp_need(int K, int L, int M, int64_t c) {
  PpNeed n;
  int64_t g = L, b = M;
  while (b) {
    const int64_t t = g % b;
    g = b;
    b = t;
  }
  n.g = (int)g;
  n.LR = L / n.g;
  n.MR = M / n.g;
  n.T = (K + L - 1) / L;
  n.rho = (int)(c % n.g);
  const int64_t c1 = c / n.g;
  n.r0 = (int)(c1 % n.LR);
  const int64_t w0 = c1 / n.LR - (n.T - 1);  // tile 0's first window sample, unaligned
  n.A = (int)floor_mod(w0, 4);
  n.xa0 = w0 - n.A;
  n.P = (n.MR % 2) ? 2 * n.LR : n.LR;
  int smax = 0;
  for (int t = 0; t < n.P; ++t) {
    const int qc = t * n.MR / n.LR;
    const int delta = (n.r0 + t * n.MR) / n.LR - qc;
    smax = std::max(smax, n.A + (qc & 1) + delta);
  }
  n.npmin = (n.T + smax + 1) / 2;
  n.UC = n.LR >= n.MR ? (int)(n.T - 1 - c / L) : -1;
  return n;
}

// The entry of chain_pp_list.h that serves the geometry, or -1.
int pp_entry(int K, int L, int M, int64_t c) {
  const PpNeed n = pp_need(K, L, M, c);
  if (n.LR > 8 || n.MR > 8) return -1;
  for (int i = 0; i < kPpCount; ++i) {
    const PpEntry& e = kPpEntries[i];
    // (an entry far wider than the call's taps would spend its FMAs on zero
    // taps: fewer taps take k_chain_gen or the two-launch chain)
    if (e.LR != n.LR || e.MR != n.MR || e.NP < n.npmin || e.NP > n.npmin + 4) continue;
    if (e.UC >= 0 ? (n.LR < n.MR || e.UC != n.UC || n.A != 0) : n.LR >= n.MR) continue;
    return i;
  }
  return -1;
}

// Floats of the generic kernel's x window for one tile: the tile's input span
// ((kGenTile-1) M / L + T), up to 3 of alignment, and taps past T reading up
// to kGenTT - T samples beyond; at least the store staging.
int gen_window(int L, int M, int T) {
  const int64_t w = ((int64_t)(kGenTile - 1) * M) / L + T + 4 + (kGenTT - T) + 2;
  const int64_t r = (w + 3) / 4 * 4;
  return (int)std::max<int64_t>(r, std::max(staging_floats(kGenTS), kScanFloats));
}

size_t gen_lds_bytes(int win) {
  return ((size_t)kGenClasses * kGenClassStride + kGenClasses + (size_t)kGenWaves * win) *
         sizeof(float);
}

int64_t gcd64(int64_t a, int64_t b) {
  while (b) {
    const int64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

// Phase classes of the generic kernel's sub-chunk starts (outputs 32 j):
// L / gcd(32 M mod L, L).
int gen_classes(int L, int M) {
  return (int)(L / gcd64(((int64_t)kGenTS * M) % L, L));
}
constexpr size_t kGenLdsMax = 64 * 1024;  // two workgroups (8 waves) per CU at least
constexpr int64_t kRepairGroups = 1024;     // workgroups of a repair kernel

size_t ct_lds_bytes(int classes, int win) {
  return ((size_t)classes * kCtClassStride + (size_t)kGenWaves * win) * sizeof(float);
}

bool tile_geometry_any(int64_t n_in, int64_t n_out, int K, int L, int M, int64_t c, int S,
                       TilePlan* tp);

// The single-pass kernels' grids are (channels or channel groups, tiles): at
// most 65535 tiles per row (201 M outputs of the L3/M2 kernel, 134 M of the
// generic ones); longer rows take the two-launch chain.
constexpr int64_t kMaxTiles = 65535;

bool tile_geometry(int64_t n_in, int64_t n_out, int K, int L, int M, int64_t c, int S,
                   TilePlan* tp) {
  return tile_geometry_any(n_in, n_out, K, L, M, c, S, tp) && tp->ntiles <= kMaxTiles;
}

bool tile_geometry_any(int64_t n_in, int64_t n_out, int K, int L, int M, int64_t c, int S,
                       TilePlan* tp) {
  // S = 0 (the EQ bypassed, or a clip-only EQ): no single-pass kernel.  z is y
  // (or its clip) there, and the two-launch chain's copy pass is cheaper than
  // the kernel's identity cascade; it also keeps the bypass's non-finite
  // semantics (an inf or NaN stays within the SRC's window; the single-pass
  // repair would carry it into every later state of the padding stages).
  if (S < 1 || S > kS || n_in < 1 || n_out < 1 || L < 1 || M < 1 || K < 1) return false;
  // n_in a multiple of 4 (the rows' float4 windows), but for the one-tap SRC
  // bypass: its x loads stop at the row's end by the buffer range check, per
  // dword (tools/probe_buffer_oob.hip), so any length runs -- one row, or
  // rows whose pitch is a multiple of 4 (launch_chain_tile checks)
  const bool one_tap = L == 1 && M == 1 && K == 1 && c == 0;
  if (n_in % 4 && !one_tap) return false;
  // SRC bypass (L = M = 1): only as the one-tap SRC (K = 1, c = 0; the
  // caller passes the tap 1.0), which the per-phase entry of the cascade alone
  // serves (chain_pp.h); any other L = M = 1 call takes the two-launch chain.
  if (L == 1 && M == 1 && (K != 1 || c != 0)) return false;
  if (n_in * 4 + 16 >= ((int64_t)1 << 31) || n_out * 4 + 16 >= ((int64_t)1 << 31)) return false;
  const int TT = (K + L - 1) / L;
  // Specialised kernel: lane windows on 16-byte boundaries, i.e. the x offset
  // of tile t's window, t*2048 + c/L - (TT-1), a multiple of 4.
  if (L == 3 && M == 2 && TT == 41 && c % L == 0 && n_out % 4 == 0 &&
      ((c / L) - (TT - 1)) % 4 == 0) {
    tp->kind = 1;
    tp->tsub = Geo3241::TSUB;
    tp->tile = Geo3241::TILE;
    tp->ntiles = ceil_div(n_out, tp->tile);
    tp->win = 0;
    return true;
  }
  // Per-phase kernels (chain_pp.h): every ratio of the app's sliders at the
  // default tap rule (and config 1's 2/1 at K = 127).
  if (L <= 64 && M <= 64) {
    const int e = pp_entry(K, L, M, c);
    if (e >= 0) {
      tp->kind = 4;
      tp->tsub = kPpEntries[e].TS;
      tp->tile = kWave * tp->tsub;
      tp->ntiles = ceil_div(n_out, tp->tile);
      tp->win = 0;
      tp->pp = e;
      return true;
    }
  }
  if (L == 160 && M == 147 && TT <= kGenTT && gen_classes(L, M) <= kGenClasses &&
      (n_out + kGenTile) * M + c < ((int64_t)1 << 31)) {
    // Window pairs up to (31 M div L) rounded to even + 10 past the lane's
    // start: at most 1 float beyond gen_window's span; +4 keeps the rounding.
    const int win = gen_window(L, M, TT) + 4;
    if (ct_lds_bytes(gen_classes(L, M), win) <= kGenLdsMax) {
      tp->kind = 3;
      tp->tsub = kGenTS;
      tp->tile = kGenTile;
      tp->ntiles = ceil_div(n_out, tp->tile);
      tp->win = win;
      return true;
    }
  }
  if (TT <= kGenTT && gen_classes(L, M) <= kGenClasses &&
      (n_out + kGenTile) * M + c < ((int64_t)1 << 31)) {
    const int win = gen_window(L, M, TT);
    if (gen_lds_bytes(win) <= kGenLdsMax) {
      tp->kind = 2;
      tp->tsub = kGenTS;
      tp->tile = kGenTile;
      tp->ntiles = ceil_div(n_out, tp->tile);
      tp->win = win;
      return true;
    }
  }
  return false;
}

size_t align256(size_t v) { return v > SIZE_MAX - 255 ? SIZE_MAX : (v + 255) & ~(size_t)255; }

// Fingerprint of everything the tables depend on that a call can state on the
// host: the kernel kind and geometry, the cascade (sos bits) and the table
// layout version.  FNV-1a, 64 bit.
uint64_t tables_key(const TilePlan& tp, int64_t n_in, int64_t n_out, int K, int L, int M,
                    int64_t c, const double* sos, int S) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&h](const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) {
      h ^= b[i];
      h *= 1099511628211ull;
    }
  };
  const int64_t v[] = {5 /* table layout version */, tp.kind, tp.tsub, tp.kind == 4 ? tp.pp : -1,
                       n_in, n_out, K, L, M, c, S,
                       (int64_t)sizeof(TileTables)};
  mix(v, sizeof(v));
  if (S > 0 && sos) mix(sos, sizeof(double) * 5 * (size_t)S);
  return h ? h : 1;  // 0 never names a table
}

// Solves the 4x4 system M z = r in place (partial pivoting); false if singular
// to working precision.
bool solve4(double M[4][4], double r[4]) {
  for (int c = 0; c < 4; ++c) {
    int piv = c;
    for (int i = c + 1; i < 4; ++i)
      if (std::fabs(M[i][c]) > std::fabs(M[piv][c])) piv = i;
    if (!(std::fabs(M[piv][c]) > 1e-13)) return false;
    if (piv != c) {
      for (int j = 0; j < 4; ++j) std::swap(M[c][j], M[piv][j]);
      std::swap(r[c], r[piv]);
    }
    for (int i = c + 1; i < 4; ++i) {
      const double f = M[i][c] / M[c][c];
      for (int j = c; j < 4; ++j) M[i][j] -= f * M[c][j];
      r[i] -= f * r[c];
    }
  }
  for (int c = 3; c >= 0; --c) {
    double s = r[c];
    for (int j = c + 1; j < 4; ++j) s -= M[c][j] * r[j];
    r[c] = s / M[c][c];
  }
  return true;
}

// Pass-1 tables in input-normal coordinates (file comment, step 2): the state
// covariance of the first n states under unit white noise, X = sum_k A^k B B^T
// A^kT (doubling: X <- X + P X P^T, P <- P^2), its Cholesky factor P (X = P
// P^T), Gc[i] = P^-1 A^(tsub-1-i) B in float32 and Q = T^-1 P.  Any
// invertible P gives the exact E' in float64 arithmetic; input-normal
// coordinates keep the float32 sums well scaled.  false when X is not
// numerically positive definite (an uncontrollable mode, e.g. a band cancelled
// by its inverse) or P is ill-conditioned: the two-launch chain serves those.
bool input_normal_tables(const std::vector<double>& A, const double* Bv,
                         const std::vector<double>& Ti, int n, int tsub, TileTables* tt) {
  if (n == 0) return true;  // no real stage: pass 1 sums nothing
  auto at = [&](const std::vector<double>& M, int r, int c) -> double { return M[(size_t)r * kD + c]; };
  std::vector<double> X((size_t)kD * kD, 0.0), Pw(A), tmp((size_t)kD * kD);
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) X[(size_t)r * kD + c] = Bv[r] * Bv[c];
  for (int it = 0; it < 40; ++it) {
    // X += Pw X Pw^T
    double pmax = 0.0;
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < n; ++c) {
        double acc = 0.0;
        for (int k = 0; k < n; ++k) acc += at(Pw, r, k) * at(X, k, c);
        tmp[(size_t)r * kD + c] = acc;
      }
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < n; ++c) {
        double acc = 0.0;
        for (int k = 0; k < n; ++k) acc += at(tmp, r, k) * at(Pw, c, k);
        X[(size_t)r * kD + c] += acc;
      }
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < n; ++c) {
        double acc = 0.0;
        for (int k = 0; k < n; ++k) acc += at(Pw, r, k) * at(Pw, k, c);
        tmp[(size_t)r * kD + c] = acc;
        pmax = std::max(pmax, std::fabs(acc));
      }
    Pw.swap(tmp);
    if (pmax < 1e-30) break;
  }
  // Cholesky X = P P^T (lower).
  std::vector<double> P((size_t)kD * kD, 0.0), Pi((size_t)kD * kD, 0.0);
  for (int j = 0; j < n; ++j) {
    double d = at(X, j, j);
    for (int k = 0; k < j; ++k) d -= at(P, j, k) * at(P, j, k);
    if (!(d > 1e-24 * at(X, j, j)) || !(d > 0.0)) return false;
    const double pj = std::sqrt(d);
    P[(size_t)j * kD + j] = pj;
    for (int i = j + 1; i < n; ++i) {
      double v = at(X, i, j);
      for (int k = 0; k < j; ++k) v -= at(P, i, k) * at(P, j, k);
      P[(size_t)i * kD + j] = v / pj;
    }
  }
  // P^-1 (lower triangular, forward substitution per column).
  for (int c = 0; c < n; ++c)
    for (int r = c; r < n; ++r) {
      double v = (r == c) ? 1.0 : 0.0;
      for (int k = c; k < r; ++k) v -= at(P, r, k) * at(Pi, k, c);
      Pi[(size_t)r * kD + c] = v / at(P, r, r);
    }
  double nP = 0.0, nPi = 0.0;
  for (int r = 0; r < n; ++r) {
    double a = 0.0, b = 0.0;
    for (int c = 0; c < n; ++c) {
      a += std::fabs(at(P, r, c));
      b += std::fabs(at(Pi, r, c));
    }
    nP = std::max(nP, a);
    nPi = std::max(nPi, b);
  }
  if (!(nP * nPi < 1e8)) return false;
  // Gc[i] = P^-1 A^(tsub-1-i) B, i = tsub-1 down to 0.
  std::vector<double> g(Bv, Bv + kD), gn(kD);
  for (int i = tsub - 1; i >= 0; --i) {
    for (int r = 0; r < kD; ++r) {
      double v = 0.0;
      for (int c = 0; c < n && r < n; ++c) v += at(Pi, r, c) * g[c];
      tt->Gc[i / 2][r][i % 2] = (float)v;
    }
    for (int r = 0; r < n; ++r) {
      double v = 0.0;
      for (int c = 0; c < n; ++c) v += at(A, r, c) * g[c];
      gn[r] = v;
    }
    for (int r = 0; r < n; ++r) g[r] = gn[r];
  }
  // Q = T^-1 P (both lower triangular).
  for (int r = 0; r < kD; ++r)
    for (int c = 0; c < kD; ++c) {
      double v = 0.0;
      if (r < n && c < n)
        for (int k = c; k <= r; ++k) v += at(Ti, r, k) * at(P, k, c);
      tt->Q[r][c] = v;
    }
  return true;
}

// Block-diagonal form of the first 2*Sr states (the real stages): T block
// unit lower triangular with A T = T D, D = diag(A_kk).  Fills the carry part
// of the tables (G' = D^(tsub-1-i) B' with B' = T^-1 B, the powers of D, T);
// false when two stages share a pole pair or T is ill-conditioned.
bool modal_tables(const SosParams& p, int Sr, int tsub, TileTables* tt) {
  const int n = 2 * Sr;
  const std::vector<double> A = state_matrix(p, kS);  // 12 x 12
  auto Aat = [&](int r, int c) { return A[(size_t)r * kD + c]; };
  std::vector<double> T((size_t)kD * kD, 0.0);
  for (int i = 0; i < n; ++i) T[(size_t)i * kD + i] = 1.0;
  for (int j = 0; j < Sr; ++j) {
    for (int i = j + 1; i < Sr; ++i) {
      // A_ii X - X A_jj = -sum_{l=j}^{i-1} A_il T_lj
      double C[2][2] = {{0, 0}, {0, 0}};
      for (int l = j; l < i; ++l)
        for (int r = 0; r < 2; ++r)
          for (int c = 0; c < 2; ++c)
            for (int q = 0; q < 2; ++q)
              C[r][c] -= Aat(2 * i + r, 2 * l + q) * T[(size_t)(2 * l + q) * kD + 2 * j + c];
      // vec (column-major): (I (x) A_ii - A_jj^T (x) I) vec(X) = vec(C)
      double M[4][4], rhs[4];
      for (int cc = 0; cc < 2; ++cc)
        for (int rr = 0; rr < 2; ++rr) {
          const int row = cc * 2 + rr;
          rhs[row] = C[rr][cc];
          for (int c2 = 0; c2 < 2; ++c2)
            for (int r2 = 0; r2 < 2; ++r2) {
              const int col = c2 * 2 + r2;
              double v = 0.0;
              if (c2 == cc) v += Aat(2 * i + rr, 2 * i + r2);
              if (r2 == rr) v -= Aat(2 * j + c2, 2 * j + cc);
              M[row][col] = v;
            }
        }
      if (!solve4(M, rhs)) return false;
      for (int cc = 0; cc < 2; ++cc)
        for (int rr = 0; rr < 2; ++rr) T[(size_t)(2 * i + rr) * kD + 2 * j + cc] = rhs[cc * 2 + rr];
    }
  }
  // T^-1 (unit lower triangular: forward substitution per column).
  std::vector<double> Ti((size_t)kD * kD, 0.0);
  for (int c = 0; c < n; ++c)
    for (int r = 0; r < n; ++r) {
      double s = (r == c) ? 1.0 : 0.0;
      for (int q = 0; q < r; ++q) s -= T[(size_t)r * kD + q] * Ti[(size_t)q * kD + c];
      Ti[(size_t)r * kD + c] = s;
    }
  double nT = 0.0, nTi = 0.0;
  for (int r = 0; r < n; ++r) {
    double a = 0.0, b2 = 0.0;
    for (int c = 0; c < n; ++c) {
      a += std::fabs(T[(size_t)r * kD + c]);
      b2 += std::fabs(Ti[(size_t)r * kD + c]);
    }
    nT = std::max(nT, a);
    nTi = std::max(nTi, b2);
  }
  if (!(nT * nTi < 1e8)) return false;
  // B of the realisation (includes the input gain), then B' = T^-1 B.
  double Bv[kD] = {0}, Bp[kD];
  cascade_state_step(p, kS, true, Bv, 1.0);
  for (int r = 0; r < kD; ++r) {
    double s = 0.0;
    for (int c = 0; c < n; ++c) s += Ti[(size_t)r * kD + c] * Bv[c];
    Bp[r] = r < n ? s : 0.0;
  }
  auto mul = [](const double* X, const double* Y, double* Z) {
    const double z0 = X[0] * Y[0] + X[1] * Y[2], z1 = X[0] * Y[1] + X[1] * Y[3];
    const double z2 = X[2] * Y[0] + X[3] * Y[2], z3 = X[2] * Y[1] + X[3] * Y[3];
    Z[0] = z0;
    Z[1] = z1;
    Z[2] = z2;
    Z[3] = z3;
  };
  for (int k = 0; k < kS; ++k) {
    double Dk[4] = {0, 0, 0, 0};
    if (k < Sr)
      for (int q = 0; q < 4; ++q) Dk[q] = Aat(2 * k + q / 2, 2 * k + q % 2);
    // G'[i] block k = D_k^(tsub-1-i) B'_k, from i = tsub-1 down.
    double g0 = Bp[2 * k], g1 = Bp[2 * k + 1];
    for (int i = tsub - 1; i >= 0; --i) {
      tt->G[i][2 * k] = g0;
      tt->G[i][2 * k + 1] = g1;
      const double n0 = Dk[0] * g0 + Dk[1] * g1, n1 = Dk[2] * g0 + Dk[3] * g1;
      g0 = n0;
      g1 = n1;
    }
    // D_k^tsub by square-and-multiply, then repeated squaring per level.
    double R[4] = {1, 0, 0, 1}, Bq[4] = {Dk[0], Dk[1], Dk[2], Dk[3]};
    for (int e = tsub; e > 0; e >>= 1) {
      if (e & 1) mul(R, Bq, R);
      if (e > 1) mul(Bq, Bq, Bq);
    }
    for (int d = 0; d < 6; ++d) {
      for (int q = 0; q < 4; ++q) tt->Dp[d][k][q] = k < Sr ? R[q] : 0.0;
      mul(R, R, R);
    }
  }
  for (int r = 0; r < kD; ++r)
    for (int c = 0; c < kD; ++c) tt->T[r][c] = (r < n && c < n) ? T[(size_t)r * kD + c] : 0.0;
  return input_normal_tables(A, Bv, Ti, n, tsub, tt);
}

// Tap pairs of the packed SRC: branch ph, pair p = (h[2p - a], h[2p + 1 - a])
// with h[u] = taps[ph + L (TT - 1 - u)] (0 outside [0, TT) or past K) and a the
// branch's window parity.
template <class GEO>
void tap_pairs(const float* taps, int K, TileTables* tt) {
  for (int p = 0; p < kNPMax; ++p)
    for (int ph = 0; ph < 4; ++ph)
      for (int e = 0; e < 2; ++e) {
        float v = 0.f;
        const int a = ph < GEO::L ? branch_parity<GEO>(ph) : -1;
        if (a >= 0 && p < GEO::NP) {
          const int u = 2 * p + e - a;
          const int k = ph + GEO::L * (GEO::TT - 1 - u);
          if (u >= 0 && u < GEO::TT && k < K) v = taps[k];
        }
        tt->TP[p][ph][e] = v;
      }
}

// Class tables of the generic kernel (TileTables::seq / adv).
void gen_sequences(const float* taps, int K, int L, int M, int64_t c, TileTables* tt) {
  const int T = (K + L - 1) / L, C = gen_classes(L, M);
  const int64_t step = ((int64_t)kGenTS * M) % L, dphi = M % L;
  for (int k = 0; k < C; ++k) {
    int64_t phi = (c % L + k * step) % L;  // branch of the class's first output
    uint32_t bits = 0;
    for (int i = 0; i < kGenTS; ++i) {
      for (int u = 0; u < kGenTT; ++u) {
        const int64_t idx = phi + (int64_t)L * (T - 1 - u);
        tt->seq[k][i][u] = (u < T && idx < K) ? taps[idx] : 0.f;
      }
      if (phi + dphi >= L) bits |= 1u << i;
      phi = (phi + dphi) % L;
    }
    tt->adv[k] = bits;
  }
  tt->classes = C;
}

// Shifted class rows of k_chain_gct (TileTables::seqs).
void ct_sequences(const float* taps, int K, int L, int M, int64_t c, TileTables* tt) {
  const int T = (K + L - 1) / L, C = gen_classes(L, M);
  const int64_t step = ((int64_t)kGenTS * M) % L;
  for (int k = 0; k < C; ++k) {
    const int64_t phi0 = (c % L + k * step) % L;  // branch of the class's first output
    for (int i = 0; i < kGenTS; ++i) {
      const int64_t g = (int64_t)i * M / L;
      const int64_t d = (phi0 + (int64_t)i * M) / L - g;  // 0 or 1
      const int64_t phi = (phi0 + (int64_t)i * M) % L;
      const int sh = (int)((g & 1) + d);
      for (int v = 0; v < kCtRow; ++v) {
        const int u = v - sh;
        const int64_t idx = phi + (int64_t)L * (T - 1 - u);
        tt->seqs[k][i][v] = (v < kCtTaps && u >= 0 && u < T && idx < K) ? taps[idx] : 0.f;
      }
    }
  }
}

// Branch 0 of the L3/M2 tile a pure delay (src_part's DLY): its tap pairs are
// zero except the centre tap's slot, which is finite and non-zero.
template <class GEO>
bool delay_branch(const TileTables* tt) {
  if (branch_parity<GEO>(0) < 0) return false;
  constexpr int sl = dly_slot<GEO>();
  for (int p = 0; p < GEO::NP; ++p)
    for (int e = 0; e < 2; ++e) {
      const float v = tt->TP[p][0][e];
      const bool centre = 2 * p + e == sl;
      if (centre ? !(std::isfinite(v) && v != 0.f) : v != 0.f) return false;
    }
  // the pairs the DLY kernel skips (void_pair) hold zero taps
  for (int p = 0; p < GEO::NP; ++p)
    for (int ph = 1; ph < GEO::L; ++ph)
      if (void_pair<GEO>(p, ph) && (tt->TP[p][ph][0] != 0.f || tt->TP[p][ph][1] != 0.f))
        return false;
  return true;
}

// Tap rows of the per-phase kernel entry e (TileTables::tpw, chain_pp.h):
// slot t's row p, e = h[2 p + e - s(t)] of its branch phi(t), h[u] = taps[phi
// + L (T - 1 - u)] (0 outside [0, T) or past K).  With a delay branch (e.UC >=
// 0) its slots' rows must hold the centre tap alone (finite, non-zero) at 2 p
// + e = UC + s(t); false otherwise (the two-launch chain serves the call).
bool pp_rows(const float* taps, int K, int L, int M, int64_t c, const PpEntry& e,
             TileTables* tt) {
  const PpNeed n = pp_need(K, L, M, c);
  if (n.P * e.NP * 2 > kPpTapFloats) return false;
  float td = 0.f;
  for (int t = 0; t < n.P; ++t) {
    const int qc = t * n.MR / n.LR;
    const int delta = (n.r0 + t * n.MR) / n.LR - qc;
    const int phi = n.g * ((n.r0 + t * n.MR) % n.LR) + n.rho;
    const int sh = n.A + (qc & 1) + delta;
    const bool dly = e.UC >= 0 && t % n.LR == 0;
    for (int v = 0; v < 2 * e.NP; ++v) {
      const int u = v - sh;
      const int64_t idx = phi + (int64_t)L * (n.T - 1 - u);
      const float h = (u >= 0 && u < n.T && idx < K) ? taps[idx] : 0.f;
      tt->tpw[t * e.NP * 2 + v] = h;
      if (dly) {
        if (v == e.UC + sh) {
          if (!(std::isfinite(h) && h != 0.f) || (td != 0.f && h != td)) return false;
          td = h;
        } else if (h != 0.f) {
          return false;
        }
      }
    }
  }
  tt->pp_td = td;
  tt->pp_np = e.NP;
  return true;
}

// Key of tables whose taps take the DLY kernel (never 0, never the plain key).
uint64_t dly_key(uint64_t base) {
  const uint64_t k = base ^ 0x9e3779b97f4a7c15ull;
  return k ? k : 2;
}

struct TileWs {
  size_t err_off, st_off, fl_off, total;
};

TileWs tile_ws(int64_t B, int64_t ntiles) {
  TileWs w;
  w.err_off = 0;  // include/dspcore.h: the workspace's first word
  w.st_off = 256;
  const size_t st = mul_sat((size_t)B, (size_t)ntiles, kD, sizeof(double));
  const size_t fl = mul_sat((size_t)B, (size_t)ntiles, sizeof(uint32_t));
  w.fl_off = st == SIZE_MAX ? SIZE_MAX : add_sat(w.st_off, align256(st));
  w.total = (fl == SIZE_MAX || w.fl_off == SIZE_MAX) ? SIZE_MAX : add_sat(w.fl_off, align256(fl));
  return w;
}

// Launch 2 of the three-launch mode (chain_tile.h, AggEntry): wave k of the
// channel's workgroup owns state block k; lane l of round r holds tile
// t = 64 r + l.  With P = D_k^(64 TS) (a tile) and e_t the aggregates, the
// entry states S_t = sum_(s<t) P^(t-1-s) e_s come from an inclusive
// Kogge-Stone over the lanes, I_l = sum_(s<=l) P^(l-s) e_(64r+s), and the
// carry C of the rounds before: S_(64r+l) = P^l C + I_(l-1), C' = P^64 C +
// I_63.  They replace the aggregates in states[] (launch 3 reads them).
__global__ __launch_bounds__(kWave * kS) void k_tile_carry(TileArgs a) {
  typedef double m2[4];  // row-major 2x2
  auto mul = [](const m2& x, const m2& y, m2& r) {
    const double r0 = fma(x[0], y[0], x[1] * y[2]), r1 = fma(x[0], y[1], x[1] * y[3]);
    const double r2 = fma(x[2], y[0], x[3] * y[2]), r3 = fma(x[2], y[1], x[3] * y[3]);
    r[0] = r0;
    r[1] = r1;
    r[2] = r2;
    r[3] = r3;
  };
  const int k = (int)threadIdx.x / kWave;
  const int lane = (int)threadIdx.x % kWave;
  const int64_t b = blockIdx.x;
  const TileTables* mt = a.tt;
  m2 pw[7];  // P^(2^j)
  {
    const m2 d5 = {mt->Dp[5][k][0], mt->Dp[5][k][1], mt->Dp[5][k][2], mt->Dp[5][k][3]};
    mul(d5, d5, pw[0]);
  }
#pragma unroll
  for (int j = 1; j < 7; ++j) mul(pw[j - 1], pw[j - 1], pw[j]);
  m2 pl = {1.0, 0.0, 0.0, 1.0};  // P^lane
#pragma unroll
  for (int j = 0; j < 6; ++j)
    if ((lane >> j) & 1) mul(pl, pw[j], pl);
  double c0 = 0.0, c1 = 0.0;
  double* st = a.states + b * a.ntiles * kD + 2 * k;
  for (int64_t t0 = 0; t0 < a.ntiles; t0 += kWave) {
    const int64_t t = t0 + lane;
    const bool in = t < a.ntiles;
    double i0 = in ? st[t * kD] : 0.0, i1 = in ? st[t * kD + 1] : 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int d = 1 << j;
      const int src = lane >= d ? lane - d : lane;
      const double x0 = shfl_f64(i0, src), x1 = shfl_f64(i1, src);
      if (lane >= d) {
        i0 = fma(pw[j][0], x0, fma(pw[j][1], x1, i0));
        i1 = fma(pw[j][2], x0, fma(pw[j][3], x1, i1));
      }
    }
    double x0 = shfl_f64(i0, lane > 0 ? lane - 1 : 0), x1 = shfl_f64(i1, lane > 0 ? lane - 1 : 0);
    if (lane == 0) x0 = x1 = 0.0;
    if (in) {
      st[t * kD] = fma(pl[0], c0, fma(pl[1], c1, x0));
      st[t * kD + 1] = fma(pl[2], c0, fma(pl[3], c1, x1));
    }
    const double j0 = shfl_f64(i0, kWave - 1), j1 = shfl_f64(i1, kWave - 1);
    const double n0 = fma(pw[6][0], c0, fma(pw[6][1], c1, j0));
    const double n1 = fma(pw[6][2], c0, fma(pw[6][3], c1, j1));
    c0 = n0;
    c1 = n1;
  }
}

// Whether a single-pass launch takes the three-launch mode: when the chained
// hand-off (~2.2 us a tile: one 441000-sample channel, 144 tiles, 0.31 ms)
// would bound it.  With t the tile's throughput cost at a full chip, chained
// ~ 2.2 us ntiles + 0.8 t B ntiles and three launches ~ 15 us + 1.4 t B
// ntiles (launch 1 redoes each tile's x, SRC, pass 1 and scan: ~0.4 t; two
// more launches).  Fitted on the cascade alone (t = 6 ns; both modes forced
// on one box at 1..4096 channels of 48000 and 441000 samples,
// profiles/r06_eq_alone_modes.txt) and checked on the SRC kernels (t = 7 ns,
// profiles/r06_three_launch_modes.txt).
bool three_launch(int64_t B, int64_t ntiles, double t_tile) {
  const double tiles = (double)B * (double)ntiles;
  return 15e-6 + 1.4 * t_tile * tiles < 2.2e-6 * (double)ntiles + 0.8 * t_tile * tiles;
}
constexpr double kTileCostIdent = 6e-9, kTileCostSrc = 7e-9;

}  // namespace

void launch_tile_carry(const TileArgs& a, int, hipStream_t s) {
  TraceScope trace("chain_tile_carry", s);
  hipLaunchKernelGGL(k_tile_carry, dim3((unsigned)a.B), dim3(kWave * kS), 0, s, a);
}

int64_t chain_tile_sub(int64_t n_in, int64_t n_out, int K, int L, int M, int64_t c, int S) {
  TilePlan tp;
  return tile_geometry(n_in, n_out, K, L, M, c, S, &tp) ? tp.tsub : 0;
}

int chain_mode(int64_t B, int64_t n_in, int64_t n_out, int K, int L, int M, int64_t c, int S) {
  TilePlan tp;
  if (B < 1 || !tile_geometry(n_in, n_out, K, L, M, c, S, &tp)) return 0;
  if (tp.kind == 4) {
    const PpEntry& e = kPpEntries[tp.pp];
    const bool ident = e.LR == 1 && e.MR == 1 && e.NP == 1 && e.UC == 0;
    if (three_launch(B, tp.ntiles, ident ? kTileCostIdent : kTileCostSrc)) return 3;
  }
  if (tp.kind != 4 && three_launch(B, tp.ntiles, kTileCostSrc)) return 3;
  return 1;
}

size_t chain_tile_workspace_bytes(int64_t B, int64_t n_in, int64_t n_out, int K, int L, int M,
                                  int64_t c, int S) {
  // The status header (256 B, word 0: hand-off status) always exists.
  TilePlan tp;
  if (B <= 0 || !tile_geometry(n_in, n_out, K, L, M, c, S, &tp)) return 256;
  return tile_ws(B, tp.ntiles).total;
}

size_t chain_tile_tables_bytes() { return sizeof(TileTables); }

int chain_tile_tables(void* out, size_t out_bytes, int64_t n_in, int64_t n_out, const float* taps,
                      int K, int L, int M, int64_t c, const double* sos, int S, uint64_t* key) {
  if (key) *key = 0;
  TilePlan tp;
  if (!tile_geometry(n_in, n_out, K, L, M, c, S, &tp)) return kNotFused;
  DSP_REQUIRE(out && out_bytes >= sizeof(TileTables), "tables buffer too small: %zu < %zu bytes",
              out_bytes, sizeof(TileTables));
  DSP_REQUIRE(taps && (S == 0 || sos), "null pointer");
  SosParams p;
  if (S > 0 && !realize(sos, S, &p)) return kNotFused;  // a b0 == 0 band: no NORM form
  if (S == 0) realize(nullptr, 0, &p);
  TileTables* tt = static_cast<TileTables*>(out);
  std::memset(tt, 0, sizeof(TileTables));
  if (!modal_tables(p, S, (int)tp.tsub, tt)) return kNotFused;  // shared poles: two-launch
  // The kernels' finite arithmetic uses the flushed taps (common.h,
  // kTapFlushRel); the caller's own taps go to the kernels' non-finite path.
  std::vector<float> ft(taps, taps + K);
  const float thr = tap_flush_threshold(taps, K, L);
  for (float& t : ft) t = flush_tap(t, thr);
  tt->flush_thr = thr;
  bool dly = false;
  if (tp.kind == 1) {
    tap_pairs<Geo3241>(ft.data(), K, tt);
    dly = delay_branch<Geo3241>(tt);
  } else if (tp.kind == 4) {
    // every entry with a delay branch needs it (no plain instantiation)
    if (!pp_rows(ft.data(), K, L, M, c, kPpEntries[tp.pp], tt)) return kNotFused;
    tt->pp_geo = tp.pp;
  } else {
    gen_sequences(ft.data(), K, L, M, c, tt);
  }
  if (tp.kind == 3) ct_sequences(ft.data(), K, L, M, c, tt);
  for (int k = 0; k < kS; ++k) {
    // NORM form (realize() above refused b0 == 0): g = 1, {c1, c2, a1, a2}
    tt->cf[k][0] = p.c[k][1];
    tt->cf[k][1] = p.c[k][2];
    tt->cf[k][2] = p.c[k][3];
    tt->cf[k][3] = p.c[k][4];
  }
  tt->gain = p.G;
  // pass 2 applies the gain at the output (pass2_cascade): states in 1 / gain
  // (Q for the float32 pass 1, G for the float64 one of the per-phase kernels)
  for (int r = 0; r < kD; ++r)
    for (int c = 0; c < kD; ++c) tt->Q[r][c] /= p.G;
  for (int i = 0; i < 64; ++i)
    for (int c = 0; c < kD; ++c) tt->G[i][c] /= p.G;
  tt->tsub = (int32_t)tp.tsub;
  tt->np = tp.kind == 1 ? Geo3241::NP : 0;
  tt->L = L;
  tt->M = M;
  tt->K = K;
  tt->S = S;
  tt->key = dly ? dly_key(tables_key(tp, n_in, n_out, K, L, M, c, sos, S))
                : tables_key(tp, n_in, n_out, K, L, M, c, sos, S);
  if (key) *key = tt->key;
  return DSP_OK;
}

int launch_chain_tile(const float* x, float* y, float* z, int64_t B, int64_t n_in, int64_t ld_x,
                      int64_t n_out, int64_t ld_y, const float* taps, int K, int L, int M,
                      int64_t c, const double* sos, int S, int clip, const void* tables,
                      uint64_t key, uint32_t max_spins, int variant, void* ws, size_t ws_bytes,
                      hipStream_t s) {
  TilePlan tp;
  if (!tables || !tile_geometry(n_in, n_out, K, L, M, c, S, &tp)) return kNotFused;
  DSP_REQUIRE(taps, "null taps");  // the non-finite path reads the caller's taps
  // Tables built for another geometry or cascade: the two-launch chain.  The
  // key also says whether the tables' taps make branch 0 a pure delay.
  const uint64_t key0 = tables_key(tp, n_in, n_out, K, L, M, c, sos, S);
  const bool dly = key == dly_key(key0);
  if (key != key0 && !dly) return kNotFused;
  // (one row: its pitch addresses nothing)
  auto aligned = [B](const void* p, int64_t ld) {
    return (B == 1 || (ld & 3) == 0) && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  };
  if (!aligned(x, ld_x) || (y && !aligned(y, ld_y)) || !aligned(z, ld_y)) return kNotFused;
  SosParams p;
  if (S > 0 && !realize(sos, S, &p)) return kNotFused;
  if (S == 0) realize(nullptr, 0, &p);
  const TileWs w = tile_ws(B, tp.ntiles);
  DSP_REQUIRE(ws && ws_bytes >= w.total, "chain workspace too small: %zu < %zu bytes", ws_bytes,
              w.total);
  DSP_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 255) == 0, "chain workspace not 256-B aligned");
  DSP_REQUIRE((reinterpret_cast<uintptr_t>(tables) & 255) == 0, "chain tables not 256-B aligned");
  DSP_REQUIRE(B * tp.ntiles < ((int64_t)1 << 31), "batch too large for one launch");
  char* base = static_cast<char*>(ws);
  TileArgs a;
  a.x = x;
  a.y = y;
  a.z = z;
  a.tt = static_cast<const TileTables*>(tables);
  a.states = reinterpret_cast<double*>(base + w.st_off);
  a.flags = reinterpret_cast<uint32_t*>(base + w.fl_off);
  a.err = reinterpret_cast<uint32_t*>(base + w.err_off);
  a.B = B;
  a.n_in = n_in;
  a.ld_x = ld_x;
  a.n_out = n_out;
  a.ld_y = ld_y;
  a.ntiles = tp.ntiles;
  a.cq = c / L;
  a.clip = clip;
  a.max_spins = max_spins;
  a.taps = taps;
  a.c = c;
  a.K = K;
  a.L = L;
  a.M = M;
  a.T = (K + L - 1) / L;
  a.win = tp.win;
  // The repair kernel after the single-pass one (k_chain_*_repair): 64
  // channels per wave, at most kRepairGroups workgroups.
  const bool one_wave = tp.kind == 1 || tp.kind == 4;  // one-wave workgroups
  const int64_t groups = one_wave ? B : ceil_div(B, (int64_t)kGenWaves);
  const int64_t rwaves = one_wave ? 1 : kGenWaves;
  const unsigned rgrid =
      (unsigned)std::min<int64_t>(ceil_div(B, kWave * rwaves), kRepairGroups);
  if (tp.kind == 4) {
    // the per-phase kernels (chain_pp_<n>.hip): tile 0's window starts at xa0
    // (a multiple of 4; the alignment A is in the tap rows)
    const PpNeed n = pp_need(K, L, M, c);
    a.cq = n.xa0;
    const PpEntry& e = kPpEntries[tp.pp];
    // the three-launch mode for small batches of long rows (variant 4 forces
    // it, 2 the chained tiles)
    const bool ident = e.LR == 1 && e.MR == 1 && e.NP == 1 && e.UC == 0;
    const bool three = variant != 2 &&
        (variant == 4 || three_launch(B, tp.ntiles, ident ? kTileCostIdent : kTileCostSrc));
    int rc = launch_chain_pp_0(e, a, rgrid, three, s);
    if (rc == kNotFused) rc = launch_chain_pp_1(e, a, rgrid, three, s);
    if (rc == kNotFused) rc = launch_chain_pp_2(e, a, rgrid, three, s);
    if (rc == kNotFused) rc = launch_chain_pp_3(e, a, rgrid, three, s);
    if (rc == kNotFused) return set_error(DSP_EINVAL, "no per-phase kernel for entry %d", tp.pp);
    return rc;
  } else if (tp.kind == 1) {
    // (No persistent variant: one measured 9 % slower at config 4 and 5 % at
    // config 3 than these chained tiles, profiles/r04_tilep_ab.txt.)
    const dim3 grid((unsigned)B, (unsigned)tp.ntiles);
    if (variant != 2 && (variant == 4 || three_launch(B, tp.ntiles, kTileCostSrc))) {
      {
        TraceScope trace("chain_tile_agg", s);
        auto k1 = dly ? k_chain_tile3<Geo3241, true, 1> : k_chain_tile3<Geo3241, false, 1>;
        hipLaunchKernelGGL(k1, grid, dim3(kWave), 0, s, a);
      }
      launch_tile_carry(a, Geo3241::TSUB, s);
      TraceScope trace("chain_tile", s);
      auto k3 = dly ? k_chain_tile3<Geo3241, true, 2> : k_chain_tile3<Geo3241, false, 2>;
      hipLaunchKernelGGL(k3, grid, dim3(kWave), 0, s, a);
    } else {
      TraceScope trace("chain_tile", s);
      auto kern = dly ? k_chain_tile<Geo3241, true> : k_chain_tile<Geo3241, false>;
      hipLaunchKernelGGL(kern, grid, dim3(kWave), 0, s, a);
    }
    TraceScope trace("chain_repair", s);
    auto rep = dly ? k_chain_tile_repair<Geo3241, true> : k_chain_tile_repair<Geo3241, false>;
    hipLaunchKernelGGL(rep, dim3(rgrid), dim3(kWave), 0, s, a);
  } else if (tp.kind == 3) {
    DSP_REQUIRE(groups * tp.ntiles < ((int64_t)1 << 31), "batch too large for one launch");
    const size_t shm = ct_lds_bytes(gen_classes(L, M), tp.win);
    auto kern = a.T <= 7 ? k_chain_gct<160, 147, true> : k_chain_gct<160, 147, false>;
    auto rep = a.T <= 7 ? k_chain_gct_repair<160, 147, true> : k_chain_gct_repair<160, 147, false>;
    auto pers = a.T <= 7 ? k_chain_gcp<160, 147, true> : k_chain_gcp<160, 147, false>;
    if (int rc = allow_lds(kern, shm)) return rc;
    if (int rc = allow_lds(rep, shm)) return rc;
    if (int rc = allow_lds(pers, shm)) return rc;
    // Persistent kernel when the batch fills the chip with whole rounds of
    // channel groups (a smaller batch runs the chained kernel, whose tiles of
    // one channel overlap everything but their carry).
    const int res = a.T <= 7 ? resident_groups<k_chain_gcp<160, 147, true>>(kWave * kGenWaves, shm)
                             : resident_groups<k_chain_gcp<160, 147, false>>(kWave * kGenWaves, shm);
    const int64_t rounds = res > 0 ? ceil_div(groups, res) : 0;
    const bool fits = tp.win <= 4 * kGcpWin * kWave && tp.win > 4 * (kGcpWin - 1) * kWave;
    // (the three-launch mode is for batches far below the persistent kernel's)
    const bool three = variant == 4 || (variant == 0 && three_launch(B, tp.ntiles, kTileCostSrc));
    const bool persistent = !three && fits && res > 0 && groups >= res &&
                            groups * 8 >= rounds * res * 7 && variant != 2;
    if (three) {
      auto k1 = a.T <= 7 ? k_chain_gct3<160, 147, true, 1> : k_chain_gct3<160, 147, false, 1>;
      auto k3 = a.T <= 7 ? k_chain_gct3<160, 147, true, 2> : k_chain_gct3<160, 147, false, 2>;
      if (int rc = allow_lds(k1, shm)) return rc;
      if (int rc = allow_lds(k3, shm)) return rc;
      {
        TraceScope trace("chain_tile_agg", s);
        hipLaunchKernelGGL(k1, dim3((unsigned)groups, (unsigned)tp.ntiles), dim3(kWave * kGenWaves),
                           shm, s, a);
      }
      launch_tile_carry(a, kGenTS, s);
      TraceScope trace("chain_tile", s);
      hipLaunchKernelGGL(k3, dim3((unsigned)groups, (unsigned)tp.ntiles), dim3(kWave * kGenWaves),
                         shm, s, a);
    } else {
      TraceScope trace("chain_tile", s);
      if (persistent || (variant == 3 && fits))
        hipLaunchKernelGGL(pers, dim3((unsigned)std::min<int64_t>(groups, std::max(res, 1))),
                           dim3(kWave * kGenWaves), shm, s, a);
      else
        hipLaunchKernelGGL(kern, dim3((unsigned)groups, (unsigned)tp.ntiles), dim3(kWave * kGenWaves),
                           shm, s, a);
    }
    TraceScope trace("chain_repair", s);
    hipLaunchKernelGGL(rep, dim3(rgrid), dim3(kWave * kGenWaves), shm, s, a);
  } else {
    DSP_REQUIRE(groups * tp.ntiles < ((int64_t)1 << 31), "batch too large for one launch");
    const size_t shm = gen_lds_bytes(tp.win);
    auto kern = M < L ? k_chain_gen<true> : k_chain_gen<false>;
    auto rep = M < L ? k_chain_gen_repair<true> : k_chain_gen_repair<false>;
    if (int rc = allow_lds(kern, shm)) return rc;
    if (int rc = allow_lds(rep, shm)) return rc;
    const dim3 grid((unsigned)groups, (unsigned)tp.ntiles);
    if (variant != 2 && (variant == 4 || three_launch(B, tp.ntiles, kTileCostSrc))) {
      auto k1 = M < L ? k_chain_gen3<true, 1> : k_chain_gen3<false, 1>;
      auto k3 = M < L ? k_chain_gen3<true, 2> : k_chain_gen3<false, 2>;
      if (int rc = allow_lds(k1, shm)) return rc;
      if (int rc = allow_lds(k3, shm)) return rc;
      {
        TraceScope trace("chain_tile_agg", s);
        hipLaunchKernelGGL(k1, grid, dim3(kWave * kGenWaves), shm, s, a);
      }
      launch_tile_carry(a, kGenTS, s);
      TraceScope trace("chain_tile", s);
      hipLaunchKernelGGL(k3, grid, dim3(kWave * kGenWaves), shm, s, a);
    } else {
      TraceScope trace("chain_tile", s);
      hipLaunchKernelGGL(kern, grid, dim3(kWave * kGenWaves), shm, s, a);
    }
    TraceScope trace("chain_repair", s);
    hipLaunchKernelGGL(rep, dim3(rgrid), dim3(kWave * kGenWaves), shm, s, a);
  }
  DSP_LAUNCHED("k_chain_tile");
  return DSP_OK;
}

}  // namespace dsp
