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

namespace dsp {
namespace {

// Cache policy of the x loads and the y/z stores: nt (streaming; every byte
// is touched once per launch).  Measured -1.6 % chain time at config 4, and
// the spectrum launch that follows runs 6 % faster.
constexpr int kStream = 2;
constexpr int kSc1 = 16;  // cache policy sc1: coherent at agent scope
constexpr int kLS = 32;  // SRC input samples per sub-chunk = lane stride in x
constexpr int kS = 6;    // stages (fewer are padded with exact identity stages)
constexpr int kD = 2 * kS;
constexpr int kNPMax = 32;  // tap pairs per polyphase branch (ceil(K/L) <= 62)
constexpr int kScanRow = 14;  // doubles per row of the blocked carry scan (12 used)
// The park row (the tile's entry state) at double 928: dword 1856, a multiple
// of 64, so lane 0's read of it shares no bank with lane 1's row 1.
constexpr int kScanPark = 928;
constexpr int kScanFloats = (kScanPark + 16) * 2;  // its LDS: 64 rows + row 64 + the park row
                                                   // (+4 doubles idle lanes read)


typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Padded LDS image of the tile's x window: 4 floats after every 32, so lane l's
// window (x offset 32 l) starts at float 36 l; the 64 lanes' ds_read_b128 then
// cover all 64 banks once per lane group and are 16-byte aligned.
__host__ __device__ constexpr int xpad(int g) { return g + 4 * (g >> 5); }

template <int L_, int M_, int TT_, int CR_>
struct TileGeo {
  static constexpr int L = L_, M = M_, TT = TT_, CR = CR_;
  static_assert((kLS * L) % M == 0, "32 input samples per sub-chunk must make whole outputs");
  static_assert(M % 2 == 0, "packed taps: windows of one branch share their x parity");
  static constexpr int TSUB = kLS * L / M;   // outputs per lane
  static constexpr int TILE = kWave * TSUB;  // outputs per workgroup
  static_assert(TSUB % 12 == 0 && TSUB <= kWave, "SRC in parts of 12; two float4 halves");
  static constexpr int NP = TT / 2 + 1;      // tap pairs per branch
  static_assert(NP <= kNPMax, "tap pairs");
  static constexpr int qi(int i) { return (i * M + CR) / L; }
  static constexpr int phi(int i) { return (i * M + CR) % L; }
  // Output i sums taps u = -a .. 2 NP - 1 - a against x[qi + u] in pairs of
  // (even, odd) x indices, a = qi mod 2: its pairs start at x index qs(i).
  static constexpr int qs(int i) { return qi(i) & ~1; }
  static constexpr int W = qs(TSUB - 1) + 2 * NP;                   // lane window
  static constexpr int NWIN = (kLS * (kWave - 1) + W + 3) / 4 * 4;  // tile window
  static constexpr int XF = xpad(NWIN + 4) + 4;                     // x image (floats)
  static constexpr int RS = TSUB + 4;                               // staging row stride
  static constexpr int SF = (kWave / 2) * RS;                       // staging (floats)
  static constexpr int CF = (kWave + 1) * kD * 2;                   // scan slots (floats)
  static constexpr int LDSF0 = XF > SF ? (XF > CF ? XF : CF) : (SF > CF ? SF : CF);
  static constexpr int LDSF = LDSF0 > kScanFloats ? LDSF0 : kScanFloats;
  static_assert(L <= 4, "four branch slots per tap pair row");
  static_assert(qs(TSUB - 1) < W, "");
};

// Per-branch x parity of the windows (-1: no output of the sub-chunk uses the
// branch); every output of a branch must share it (M even makes it so).
template <class GEO>
constexpr int branch_parity(int ph) {
  int a = -1;
  for (int i = 0; i < GEO::TSUB; ++i)
    if (GEO::phi(i) == ph) {
      const int ai = GEO::qi(i) & 1;
      if (a >= 0 && a != ai) return -2;
      a = ai;
    }
  return a;
}

// Generic kernel geometry (k_chain_gen, below).
constexpr int kGenTS = 32;                    // outputs per lane
constexpr int kGenTile = kWave * kGenTS;      // outputs per tile (wave)
constexpr int kGenWaves = 4;                  // waves (channels) per workgroup
constexpr int kGenTT = 8;                     // taps per output row (T <= 8)
constexpr int kGenClasses = 8;                // max sub-chunk phase classes
constexpr int kGenClassStride = kGenTS * kGenTT + 4;  // LDS floats per class (+4: bank spread)
// Select-free variant for a compile-time ratio (k_chain_gct<L, M>, below).
constexpr int kCtTaps = 10;   // tap slots per output: T <= 8 taps shifted by 0..2
constexpr int kCtRow = 12;    // floats per output row (b128 + b128 + b64 reads)
constexpr int kCtClassStride = kGenTS * kCtRow + 4;  // 388: class rows on distinct bank quads

// Tables of the single-pass kernel, built on the host in float64
// (dsp_chain_tile_tables) and read by the kernel through the scalar cache.
struct TileTables {
  uint64_t key;            // dsp_chain_tile_tables' fingerprint of what they were built for
  double G[64][kD];        // G'[i] = T^-1 A^(TSUB-1-i) B, i < TSUB (block-diagonal coords)
  float Gc[32][kD][2];     // Gc[j][d] = rows 2j, 2j+1 of P^-1 A^(TSUB-1-i) B (input-normal), float32
  double Q[kD][kD];        // T^-1 P, lower triangular (input-normal -> block-diagonal)
  double Dp[6][kS][4];     // D_k^(TSUB 2^d), row-major 2x2, d = 0..5
  double T[kD][kD];        // s = T m (row-major; zero rows/cols: padding stages)
  float TP[kNPMax][4][2];  // tap pairs: TP[p][ph] = (h[2p - a_ph], h[2p + 1 - a_ph])
  int32_t tsub, np, L, M, K, S;  // what the tables were built for (in `key`)
  // The DF2 realisation (cascade.h, NORM form): per stage {c1, c2, a1, a2}
  // and the input gain.  Read through the scalar cache right where pass 2
  // needs them instead of occupying ~50 SGPRs as kernel arguments for the
  // whole kernel (which made the compiler spill SGPRs to VGPR lanes).
  double cf[kS][4];
  double gain;
  // Generic kernel: sub-chunks start at outputs m = 32 j, whose polyphase
  // branch (32 j M + c) mod L takes `classes` values (class of j: j mod
  // classes).  seq[k][i] = the taps of output i of a class-k sub-chunk (u < T,
  // zero beyond); bit i of adv[k] = 1 when q advances by M div L + 1 (not
  // M div L) from output i to i + 1.
  float seq[kGenClasses][kGenTS][kGenTT];
  uint32_t adv[kGenClasses];
  int32_t classes, pad;
  // k_chain_gct<L, M>: the same class rows with the lane's window offset
  // folded in.  Output i of a class-k sub-chunk reads the window pairs from
  // (i M div L) rounded down to even; seqs[k][i][v] = h[v - s_i] with the
  // shift s_i = (i M div L) mod 2 + (1 if the class's phase carries q one
  // further, else 0), zero outside the T taps.
  alignas(16) float seqs[kGenClasses][kGenTS][kCtRow];
  // Largest flushed |tap| (common.h, kTapFlushRel), for the non-finite path.
  float flush_thr;
  int32_t pad3[3];
};

struct TileArgs {
  const float* x;
  float* y;
  float* z;
  const TileTables* tt;     // device copy of dsp_chain_tile_tables' output
  double* states;           // [B][ntiles][12] tile end states (block-diagonal coords)
  uint32_t* flags;          // [B][ntiles]
  uint32_t* err;            // workspace status word: set when a hand-off wait gave up
  int64_t B, n_in, ld_x, n_out, ld_y, ntiles, cq;
  int clip;
  uint32_t max_spins;       // polls before a hand-off wait gives up
  // generic kernel (k_chain_gen) only
  const float* taps;        // device taps [K]
  int64_t c;                // 'same' offset of the expanded convolution
  int K, L, M, T, win;      // win: floats of one wave's x window
};

__device__ __forceinline__ void fence() { asm volatile("" ::: "memory"); }

// The lane's index in its wave, recomputed (mbcnt): late uses of threadIdx.x
// would keep its VGPR live through the whole kernel.
__device__ __forceinline__ int lane_id() {
  return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Pins v[0..N) at this point of the program: the values are computed before it
// and later uses start after it.  Keeps the scheduler from overlapping phases
// whose live registers together exceed the 128 VGPRs of 4 waves per SIMD.
template <int N, class T>
__device__ __forceinline__ void pin(T (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

// 2x2 block of v <- M v + acc (M row-major; any address space).
template <class PTR>
__device__ __forceinline__ void mac2(PTR M, double x0, double x1, double& a0, double& a1) {
  a0 = fma(M[0], x0, fma(M[1], x1, a0));
  a1 = fma(M[2], x0, fma(M[3], x1, a1));
}

__device__ __forceinline__ double shfl_up_f64(double v, int d) {
  // ds_bpermute (the LDS crossbar, no LDS memory): lane l reads lane l - d.
  const int src = ((int)threadIdx.x - d) << 2;
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// ds_bpermute of a double from lane src.
__device__ __forceinline__ double shfl_f64(double v, int src) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Agent-scope hand-off accesses: global (never flat) loads/stores with sc1.
__device__ __forceinline__ uint32_t load_flag(const uint32_t* p) {
  return __hip_atomic_load((const __attribute__((address_space(1))) uint32_t*)p,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_flag(uint32_t* p, uint32_t v) {
  __hip_atomic_store((__attribute__((address_space(1))) uint32_t*)p, v,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_state(const double* p) {
  return __hip_atomic_load((const __attribute__((address_space(1))) double*)p,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_state(double* p, double v) {
  __hip_atomic_store((__attribute__((address_space(1))) double*)p, v,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

typedef __attribute__((address_space(4))) const TileTables* tt_ptr;

// SRC outputs H0 .. H0+NH-1 of the lane's sub-chunk from its window at xw
// (padded LDS image), two taps per v_pk_fma_f32: output i keeps the partial
// sums of its even- and odd-indexed x samples in the halves of one register
// pair, pairs p ascending, and y = even + odd -- the summation order of
// k_src_reg's packed path (src_poly.hip), so y is bitwise the SRC kernel's.
// DLY: branch 0's taps are zero but for its centre tap u = TT / 2 (the
// caller's taps with the sinc-zero noise flushed, common.h kTapFlushRel;
// dsp_chain_tile_tables checks it and marks the key): its outputs, every L-th,
// are that tap times one sample -- one multiply instead of NP packed FMAs, and
// for a finite window bitwise what the FMA chain gives on these taps (t x
// rounded once; the zero taps add signed zeros).  A window with an inf or NaN
// (0 * inf = NaN in the chain, not here) is rerun by the repair kernel with
// the reference's semantics (tile_cascade).  Outputs of other branches are
// unchanged.
template <class GEO>
constexpr bool dly_out(int i) { return GEO::phi(i) == 0; }
// DLY also skips the tap pairs that lie wholly outside the reference's
// default filter (K = 40 L + 1 taps; branch 1's first pair at L3/M2): both
// of their taps are zero in every table with the DLY key (delay_branch).
template <class GEO>
constexpr bool void_pair(int p, int ph) {
  const int a = branch_parity<GEO>(ph);
  if (a < 0) return true;
  for (int e = 0; e < 2; ++e) {
    const int u = 2 * p + e - a;
    if (u >= 0 && u < GEO::TT && ph + GEO::L * (GEO::TT - 1 - u) < 40 * GEO::L + 1) return false;
  }
  return true;
}
// ... as a table, so that the unrolled SRC loops index a constant (a call
// there was left to run time).
struct VoidPairs {
  bool v[kNPMax][4];
};
template <class GEO>
constexpr VoidPairs void_pairs() {
  VoidPairs t{};
  for (int p = 0; p < kNPMax; ++p)
    for (int ph = 0; ph < 4; ++ph) t.v[p][ph] = ph < GEO::L && p < GEO::NP && void_pair<GEO>(p, ph);
  return t;
}
template <class GEO>
constexpr int dly_slot() { return GEO::TT / 2 + (branch_parity<GEO>(0) > 0 ? 1 : 0); }

template <class GEO, int H0, int NH, bool DLY = false>
__device__ __forceinline__ void src_part(const float* xw, tt_ptr tt, float (&y)[GEO::TSUB]) {
  static constexpr VoidPairs kVoid = void_pairs<GEO>();
  constexpr int V0 = GEO::qs(H0) / 4 * 4;
  constexpr int V1 = GEO::qs(H0 + NH - 1) + 2 * GEO::NP;
  constexpr int NV = (V1 - V0 + 3) / 4 * 4;
  f32x2 w[NV / 2];
#pragma unroll
  for (int k = 0; k < NV / 4; ++k) {
    const f32x4 f = *reinterpret_cast<const f32x4*>(xw + xpad(V0 + 4 * k));
    w[2 * k] = f32x2{f.x, f.y};
    w[2 * k + 1] = f32x2{f.z, f.w};
  }
  f32x2 acc[NH];
#pragma unroll
  for (int i = 0; i < NH; ++i) acc[i] = f32x2{0.f, 0.f};
#pragma unroll
  for (int p = 0; p < GEO::NP; ++p) {
    // Load each pair's taps right before its FMAs (an opaque table pointer per
    // pair keeps the compiler from hoisting all 126 tap SGPRs of a part).
    tt_ptr tq = tt;
    asm volatile("" : "+s"(tq));
    f32x2 t[GEO::L];
#pragma unroll
    for (int ph = 0; ph < GEO::L; ++ph) t[ph] = f32x2{tq->TP[p][ph][0], tq->TP[p][ph][1]};
#pragma unroll
    for (int i = 0; i < NH; ++i)
      if (!(DLY && (dly_out<GEO>(H0 + i) || kVoid.v[p][GEO::phi(H0 + i)])))
        acc[i] = __builtin_elementwise_fma(t[GEO::phi(H0 + i)],
                                           w[(GEO::qs(H0 + i) - V0) / 2 + p], acc[i]);
  }
  float td = 0.f;
  if (DLY) {
    tt_ptr tq = tt;
    asm volatile("" : "+s"(tq));
    td = tq->TP[dly_slot<GEO>() / 2][0][dly_slot<GEO>() % 2];
  }
#pragma unroll
  for (int i = 0; i < NH; ++i) {
    if (DLY && dly_out<GEO>(H0 + i)) {
      const f32x2 xv = w[(GEO::qs(H0 + i) - V0) / 2 + dly_slot<GEO>() / 2];
      y[H0 + i] = td * (dly_slot<GEO>() % 2 ? xv.y : xv.x);
    } else {
      y[H0 + i] = acc[i].x + acc[i].y;
    }
  }
}

// LDS float of output float g = 4 (lane + 64 k) in store_tile's staging, as a
// per-lane base plus a constant:
//   TS = 32 (round 5): row stride 32 with the float4 column XOR-swizzled by
//            the row's low 3 bits: row r = g div 32 = lane div 8 + 8 k, column
//            4 ((lane mod 8) ^ (r mod 8)) = 4 ((lane mod 8) ^ (lane div 8 mod
//            8)): one base and 256 k;
//   TS = 48: g + 4 (g div TS) (row stride TS + 4): (lane + 64 k) div 12 = a +
//            [k >= 3] + [r + 4 (k mod 3) >= 12] with lane = 12 a + r, so three
//            bases, by k mod 3, and 276 k + 4 [k >= 3].
template <int TS>
struct StageBase {
  int b[3];
  __device__ __forceinline__ explicit StageBase(int lane) {
    if constexpr (TS == 32) {
      b[0] = 32 * (lane >> 3) + 4 * ((lane & 7) ^ ((lane >> 3) & 7));
    } else {
      static_assert(TS == 48, "staging rows of 8 or 12 float4s");
      const int a = (lane * 43) >> 9;  // lane div 12 (lane < 64)
      const int r = lane - 12 * a;
      b[0] = 4 * lane + 4 * a;
      b[1] = b[0] + 4 * ((r + 8) >> 4);   // + 4 [r >= 8]
      b[2] = b[0] + 4 * ((r + 12) >> 4);  // + 4 [r >= 4]
    }
  }
  __device__ __forceinline__ int at(int k) const {
    if constexpr (TS == 32) return b[0] + 256 * k;
    else return b[k % 3] + 276 * k + (k >= 3 ? 4 : 0);
  }
};

// Stores the tile's 64 x TS outputs (lane l holds outputs l*TS + i) as
// coalesced float4s through `rs`, a buffer resource whose base is the tile's
// first output: each half of the lanes writes its rows into LDS, then all 64
// lanes store the half's contiguous 32*TS floats.  The resource checks every
// dword: stores past the row's end are dropped, a float4 across it keeps its
// head.  TS = 48 (config 3/4): row stride TS + 4, conflict-free ds_write_b128;
// the reads take 2-way bank conflicts in some ds_read_b128 lane groups, 48
// cycles per call; an XOR-swizzled unpadded layout free of them cost more in
// the VALU that computes its addresses than the LDS cycles it saved there
// (chain 5.73-5.77 vs 5.68-5.70 ms at config 4, same box, round 4: that kernel
// is VALU-issue-bound at the power cap).  TS = 32 (round 5): the swizzle of
// StageBase, free of conflicts both ways (tools/ldsmodel.py --ts32: the padded
// layout's reads took 32 extra cycles per call) for 8 VALU per call.
template <int TS>
__device__ __forceinline__ void store_tile(float* lds, const float (&v)[TS], int lane,
                                           __amdgpu_buffer_rsrc_t rs) {
  constexpr int RS = TS == 32 ? 32 : TS + 4;
  constexpr int NF4 = (kWave / 2) * TS / 4;
  static_assert(NF4 % kWave == 0, "whole float4 rounds per half");
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const StageBase<TS> sb(lane);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    fence();
    if ((lane >> 5) == h) {
      float* row = lds + (lane & 31) * RS;
      const int sw = TS == 32 ? (lane & 7) : 0;  // the row's column swizzle
#pragma unroll
      for (int k = 0; k < TS / 4; ++k)
        *reinterpret_cast<float4*>(row + 4 * (k ^ sw)) =
            make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
    fence();
#pragma unroll
    for (int k = 0; k < NF4 / kWave; ++k) {
      // output float g = 4 (lane + 64 k) sits in row r = g div TS at r RS + g
      // mod TS = g + 4 r (StageBase)
      const int g = 4 * (lane + kWave * k);
      const float4 f = *reinterpret_cast<const float4*>(lds + sb.at(k));
      u32x4 d;
      d.x = __float_as_uint(f.x);
      d.y = __float_as_uint(f.y);
      d.z = __float_as_uint(f.z);
      d.w = __float_as_uint(f.w);
      __builtin_amdgcn_raw_buffer_store_b128(d, rs, (h * (kWave / 2) * TS + g) * 4, 0, kStream);
    }
  }
  fence();
}

// Entry state of a tile > 0: lane 0 waits for the previous tile of the
// channel (hand-off, file comment) and loads its end state into m_in (the
// other lanes leave m_in unset).
__device__ __forceinline__ void tile_entry_state(const TileArgs& a, int64_t b, int64_t tile,
                                                 int lane, double (&m_in)[kD]) {
  if (lane == 0) {
    const int64_t prev = b * a.ntiles + tile - 1;
    uint32_t spins = 0;
    bool ok = true;
    while (load_flag(a.flags + prev) == 0u) {
      if (++spins > a.max_spins) {
        // Give up: mark the status word; the flag stays for the workspace
        // reset (a late producer would set it again anyway).
        store_flag(a.err, 1u);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    fence();
#pragma unroll
    for (int d = 0; d < kD; ++d) m_in[d] = load_state(a.states + prev * kD + d);
    if (ok) store_flag(a.flags + prev, 0u);  // consumed: leave the array clear
  }
}

// LDS floats store_tile<TS> stages through.
__host__ __device__ constexpr int staging_floats(int ts) { return (kWave / 2) * (ts + 4); }

__device__ __forceinline__ void pass1_basis(tt_ptr mt, const f32x2 (&e2)[kD], double (&v)[kD]);

// Pass 1 (file comment, step 2): the sub-chunk's zero-state end state in
// block-diagonal coordinates, E' = Q sum_i Gc[i] y[i] (float32 sums in
// input-normal coordinates, one float64 change of basis).
template <int TS>
__device__ __forceinline__ void pass1_state(tt_ptr mt, const float (&y)[TS], double (&v)[kD]) {
  {
    // float32 sums in input-normal coordinates: component d keeps the sums
    // over even and odd samples in the halves of one v_pk_fma_f32 chain
    // (samples 2j, 2j+1 against the row pair Gc[j][d]) ...
    f32x2 e2[kD];
#pragma unroll
    for (int d = 0; d < kD; ++d) e2[d] = f32x2{-0.f, -0.f};  // (-0: the first FMA is a multiply)
#pragma unroll
    for (int j = 0; j < TS / 2; ++j) {
      // Each row pair's 24 floats are scalar-loaded right before its FMAs (an
      // opaque table pointer per pair keeps the compiler from hoisting the
      // whole table into SGPRs, which spills).
      tt_ptr tq = mt;
      asm volatile("" : "+s"(tq));
      const f32x2 u = f32x2{y[2 * j], y[2 * j + 1]};
#pragma unroll
      for (int d = 0; d < kD; ++d)
        e2[d] = __builtin_elementwise_fma(f32x2{tq->Gc[j][d][0], tq->Gc[j][d][1]}, u, e2[d]);
    }
    pin(e2);
    pass1_basis(mt, e2, v);
  }
}

// Pass 1's change of basis: E' = Q e in float64, e = the input-normal sums.
__device__ __forceinline__ void pass1_basis(tt_ptr mt, const f32x2 (&e2)[kD], double (&v)[kD]) {
  {
    f32x2 e[kS];
#pragma unroll
    for (int k = 0; k < kS; ++k)
      e[k] = f32x2{e2[2 * k].x + e2[2 * k].y, e2[2 * k + 1].x + e2[2 * k + 1].y};
    // ... then E' = Q e in float64 (Q lower triangular; rows from the last,
    // so that e_r dies after row r: 12 doubles live, not 24).
    double ed[kD];
#pragma unroll
    for (int k = 0; k < kS; ++k) {
      ed[2 * k] = (double)e[k].x;
      ed[2 * k + 1] = (double)e[k].y;
    }
#pragma unroll
    for (int r = kD - 1; r >= 0; --r) {
      tt_ptr tq = mt;
      asm volatile("" : "+s"(tq));
      double acc = tq->Q[r][0] * ed[0];
#pragma unroll
      for (int c = 1; c <= r; ++c) acc = fma(tq->Q[r][c], ed[c], acc);
      v[r] = acc;
    }
  }
}

// Pass 2 (file comment, step 5): DF2 entry state s = T m, the cascade rerun
// over the sub-chunk from it and the clip; y becomes z in place.
// NANCLIP: the clip keeps NaN (v_maximum3/v_minimum3, as np.clip); else one
// v_med3_f32, which may drop a NaN -- the single-pass kernels' z is finite
// wherever the repair kernel does not rerun it (tile_cascade).
template <int TS, bool NANCLIP>
__device__ __forceinline__ void pass2_cascade(const TileArgs& a, tt_ptr mt, float (&y)[TS],
                                              const double (&m)[kD]) {
  // s = T m: T is block unit lower triangular (identity diagonal blocks, zero
  // rows and columns for padding stages), so row r starts from m[r].
  double s1[kS], s2[kS];
#pragma unroll
  for (int r = 0; r < kD; ++r) {
    double acc = m[r];
#pragma unroll
    for (int cc = 0; cc < (r / 2) * 2; ++cc) acc = fma(mt->T[r][cc], m[cc], acc);
    if (r & 1) s2[r / 2] = acc;
    else s1[r / 2] = acc;
  }
  // Pass 2, diagonally pipelined: step s runs stage k on sample s - k, so the
  // six stage updates of a step are independent (six FMA chains in flight
  // instead of one 24-deep chain per sample).  Per sample and stage the
  // operations are cascade_step's: the results are bitwise the same.
  float lo = a.clip ? -1.f : -INFINITY, hi = a.clip ? 1.f : INFINITY;
  // Opaque uniform bounds: otherwise the compiler clips to +-1 and selects the
  // unclipped value per sample (4 VALU per sample instead of max + min).
  asm volatile("" : "+v"(lo), "+v"(hi));
  // The realisation's input gain prod(b0) moves to the output, after the
  // float32 conversion: the recursion runs on y with every state scaled by
  // 1 / gain (the tables' Q carries the 1 / gain, so the carry and the entry
  // states are in those coordinates), and z = fl32(v) * gain32 -- one float32
  // multiply per sample instead of a float64 one (two roundings: <= 1.5 ulp).
  const float g32 = (float)mt->gain;
  {
    double pend[kS];  // pend[k]: stage k's output from the previous step
#pragma unroll
    for (int st = 0; st < TS + kS - 1; ++st) {
#pragma unroll
      for (int k = kS - 1; k >= 0; --k) {
        const int t = st - k;
        if (t < 0 || t >= TS) continue;
        const double u = k == 0 ? (double)y[t] : pend[k - 1];
        const double c1 = mt->cf[k][0], c2 = mt->cf[k][1], a1 = mt->cf[k][2], a2 = mt->cf[k][3];
        const double w = fma(-a2, s2[k], fma(-a1, s1[k], u));
        const double v2 = fma(c2, s2[k], fma(c1, s1[k], w));
        s2[k] = s1[k];
        s1[k] = w;
        if (k == kS - 1)
          y[t] = NANCLIP ? clip_f32((float)v2 * g32, lo, hi)
                         : __builtin_amdgcn_fmed3f((float)v2 * g32, lo, hi);
        else pend[k] = v2;
      }
    }
  }
}

// Rare path of a tile with non-finite input (tile_cascade): every output of
// the lane through window_sums / nf_fix (sums(i, nf, fin) gives output i's),
// then the lane's E': NaN if its y holds an inf or NaN, else pass 1 rerun on
// the fixed y (a zero tap's NaN may have been all there was).  The outputs
// wait in the tile's own z outputs (z0: output 0 of the lane; pass 2
// overwrites them), and the loops over them are rolled: unrolled over
// registers or staged in a private array, this code cost the hot path
// registers (VGPR and SGPR spills, the scratch setup's SGPRs).
template <int TS, class SUMS>
__device__ __forceinline__ void fix_outputs(const TileArgs& a, tt_ptr mt, int64_t b, int64_t z0,
                                            float (&y)[TS], double (&v)[kD], SUMS&& sums) {
  const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(
      a.z + b * a.ld_y, 0, (int)(a.n_out * 4), 0x00020000);
  const int off0 = (int)(z0 * 4);  // outputs past n_out: dropped / read as 0, never stored
  auto get = [&](int i) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rz, off0 + 4 * i, 0, 1));
  };
  auto put = [&](int i, float f) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(f), rz, off0 + 4 * i, 0, 0);
  };
#pragma unroll
  for (int i = 0; i < TS; ++i) put(i, y[i]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bool any = false;
#pragma unroll 1
  for (int i = 0; i < TS; ++i) {
    float nf, fin, f = get(i);
    sums(i, nf, fin);
    any |= nf_fix(f, nf, fin);
    put(i, f);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (any) {
#pragma unroll
    for (int d = 0; d < kD; ++d) v[d] = __builtin_nan("");
  } else {
    // pass1_state's sums in its order (bitwise the same E'), rolled
    f32x2 e2[kD];
#pragma unroll
    for (int d = 0; d < kD; ++d) e2[d] = f32x2{0.f, 0.f};
#pragma unroll 1
    for (int j = 0; j < TS / 2; ++j) {
      const f32x2 u = f32x2{get(2 * j), get(2 * j + 1)};
#pragma unroll
      for (int d = 0; d < kD; ++d)
        e2[d] = __builtin_elementwise_fma(f32x2{mt->Gc[j][d][0], mt->Gc[j][d][1]}, u, e2[d]);
    }
    pass1_basis(mt, e2, v);
  }
#pragma unroll
  for (int i = 0; i < TS; ++i) y[i] = get(i);
}

// Steps 2-5 of the tile (file comment) for a wave that holds its y sub-chunk:
// pass 1, entry state (hand-off) and scan, publish, y out, s = T m, pass 2,
// z out.  lds: at least staging_floats(TS) floats the wave may overwrite; the
// x window there stays intact until pass 1 is done.
//
// Non-finite input.  Every x sample of a lane's window meets an FMA of some
// output of the lane whose polyphase branch is not the pure delay (flushed
// taps included: 0 * inf = NaN), so a window holding an inf or NaN leaves a
// non-finite y, E' and (fma by any finite coefficient keeps it non-finite)
// end state of the tile, and of every later tile of the channel.  The
// single-pass kernels do nothing about it; every tile publishes its end state,
// the channel's last one included, and the repair kernel that follows them
// (k_chain_*_repair) reruns a channel whose last end state is not finite from
// its first tile with a non-finite end state on.  There REPAIR tiles whose
// pass-1 state is not finite (one class test per lane, a wave ballot) call
// on_nf(y, v), which recomputes y with the reference's non-finite semantics
// (fix_outputs: window_sums / nf_fix; finite windows keep the canonical sums,
// recomputed from the window with its infs and NaNs zeroed, since the packed
// FMAs of a neighbouring output may have picked one up through a zero tap),
// reruns pass 1 on the fixed y and makes E' NaN for a lane whose y holds an
// inf or NaN (as nf_poison: every later output of the channel is NaN, as in
// the reference's cascade).
// Where a tile's entry state comes from.  ChainedEntry: the previous tile's
// workgroup (the hand-off above).  RegCarry (persistent kernels, which run the
// tiles of a channel in order in one wave): registers -- the previous tile's
// end state as its scan left it, block kb of it in each worker lane of
// segment 7 (tile_cascade stores it to the park row and refreshes it).
struct ChainedEntry {};
struct RegCarry {
  double c0, c1;
};
// k_chain_tile: the hand-off flag was polled when the tile started and, if
// it was already raised, the state went into the LDS slot `slot` by an
// agent-scope LDS-DMA behind the SRC and pass 1 (chain_tile_body); else the
// chained wait as above.
struct EarlyEntry {
  bool early;
  const double* slot;
};

template <int TS, bool YST = true, bool REPAIR = false, class ONNF, class ENTRY = ChainedEntry>
__device__ __forceinline__ void tile_cascade(const TileArgs& a, tt_ptr mt, float* lds,
                                             float (&y)[TS], int lane, int64_t b, int64_t tile,
                                             int64_t m0, ONNF&& on_nf, ENTRY&& entry = ENTRY{}) {
  constexpr bool kRegCarry = std::is_same_v<std::decay_t<ENTRY>, RegCarry>;
  constexpr bool kEarly = std::is_same_v<std::decay_t<ENTRY>, EarlyEntry>;
  // ---- 2. pass 1: zero-state end state of the sub-chunk
  double v[kD];
  pass1_state<TS>(mt, y, v);
  if constexpr (REPAIR) {
    if (__builtin_amdgcn_ballot_w64(!__builtin_isfinite(v[kD - 1]))) on_nf(y, v);  // wave-uniform
  }
  // Keep the SRC and pass 1 ahead of the hand-off wait (the compiler would
  // otherwise sink them past it).
  pin(v);

  // ---- 3. entry state of the tile and the scan across the lanes
  // Blocked scan through LDS.  Rows r = 0..63 take E'_r (row stride kScanRow
  // doubles: the b128 accesses of 16 lanes hit 16 distinct bank quads); 48
  // worker lanes, one per (state block k, segment s of 8 rows), run the
  // segment's local recurrence u <- D u + E' (D = D_k^TSUB, per-lane loads);
  // a 3-level Kogge-Stone over the 8 segments of a block (ds_bpermute, powers
  // D^(8 TSUB 2^d) by squaring D^(8 TSUB)) gives each segment its entry state;
  // each worker reruns its segment from that state and writes v_r to row r + 1,
  // so row l holds lane l's entry state m_l = v_(l-1) and the park row m_in
  // (the tile's entry state, which enters segment 0 as "segment -1").  Per
  // lane: 7 + 3 + 8 block steps and two 2x2 squarings (~80 fp64 ops), 29 b128
  // LDS accesses and 16 bpermutes, against round 2's 6 levels x 12 doubles
  // (144 FMAs + a 24-FMA entry fold, 168 bpermutes).
  typedef double f64x2 __attribute__((ext_vector_type(2)));
  double* rows = reinterpret_cast<double*>(lds);
  double* park = rows + kScanPark;
  static_assert(kScanPark >= 65 * kScanRow, "park row past the scan rows");
#pragma unroll
  for (int k = 0; k < kS; ++k)
    *reinterpret_cast<f64x2*>(rows + lane * kScanRow + 2 * k) = f64x2{v[2 * k], v[2 * k + 1]};
  // The tile's entry state (hand-off wait; lane 0) goes to the park row
  // (tile 0: zeros, one zero register pair for all six stores).
  if (tile == 0) {
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < kS; ++k) *reinterpret_cast<f64x2*>(park + 2 * k) = f64x2{0.0, 0.0};
    }
  } else if constexpr (kRegCarry) {
    // segment 7's lanes hold the previous tile's end state, block lane & 7
    // (lanes 62, 63: the park row's unused slots 12..15)
    if ((lane >> 3) == 7)
      *reinterpret_cast<f64x2*>(park + 2 * (lane & 7)) = f64x2{entry.c0, entry.c1};
  } else {
    bool got = false;
    if constexpr (kEarly) {
      if (entry.early) {
        // the state is in the LDS slot once the wave's only vector memory
        // operation in flight, the LDS-DMA, is done
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
#pragma unroll
          for (int k = 0; k < kS; ++k)
            *reinterpret_cast<f64x2*>(park + 2 * k) =
                *reinterpret_cast<const f64x2*>(entry.slot + 2 * k);
          store_flag(a.flags + b * a.ntiles + tile - 1, 0u);  // consumed
        }
        got = true;
      }
    }
    if (!got) {
      double m_in[kD];
      tile_entry_state(a, b, tile, lane, m_in);
      if (lane == 0) {
#pragma unroll
        for (int d = 0; d < kD; ++d) park[d] = m_in[d];
      }
    }
  }
  fence();
  // worker (k, s): lane 8 s + k, k < 6 (lanes 8 s + 6, 8 s + 7 idle: they
  // read the row's padding slot and the next row's first slot, so that the
  // 8 lanes of a segment cover 32 consecutive dwords; their results are never
  // stored).  With this order the b128 row accesses are free of bank
  // conflicts: a ds_write_b128 group of 8 contiguous lanes is one segment's 6
  // blocks, and the ds_read_b128 groups of 16 lanes mix two segments of each
  // parity on disjoint bank quads (MI355X_MICROARCH.md §LDS; round 3's idle
  // lanes read block 0 of their rows: 32 conflict cycles per wave).
  const int sg = lane >> 3;
  const bool worker = (lane & 7) < 6;
  // (idle lanes load the tables of "blocks" 6 and 7 too: entries of Dp's next
  // rows, in bounds, never used for a stored value)
  const int kb = lane & 7;
  const __attribute__((address_space(1))) double* Dg =
      (const __attribute__((address_space(1))) double*)&mt->Dp[0][kb][0];
  const f64x2 d0a = *reinterpret_cast<const __attribute__((address_space(1))) f64x2*>(Dg);
  const f64x2 d0b = *reinterpret_cast<const __attribute__((address_space(1))) f64x2*>(Dg + 2);
  f64x2 e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    e[i] = *reinterpret_cast<const f64x2*>(rows + (8 * sg + i) * kScanRow + 2 * kb);
  const __attribute__((address_space(1))) double* D8g = Dg + 3 * kS * 4;  // Dp[3][kb]
  f64x2 p8a = *reinterpret_cast<const __attribute__((address_space(1))) f64x2*>(D8g);
  f64x2 p8b = *reinterpret_cast<const __attribute__((address_space(1))) f64x2*>(D8g + 2);
  double u0 = e[0].x, u1 = e[0].y;
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    const double n0 = fma(d0a.x, u0, fma(d0a.y, u1, e[i].x));
    const double n1 = fma(d0b.x, u0, fma(d0b.y, u1, e[i].y));
    u0 = n0;
    u1 = n1;
  }
  // m_in (parked above) enters as segment -1: u_0 += D^(8 TSUB) m_in, and
  // segment 0's entry state is m_in.
  f64x2 mi = f64x2{0.0, 0.0};
  if (sg == 0) {
    mi = *reinterpret_cast<const f64x2*>(park + 2 * kb);
    u0 = fma(p8a.x, mi.x, fma(p8a.y, mi.y, u0));
    u1 = fma(p8b.x, mi.x, fma(p8b.y, mi.y, u1));
  }
#pragma unroll
  for (int lv = 0; lv < 3; ++lv) {
    const int dd = 1 << lv;
    const int ss = sg - dd;
    const int src = ss >= 0 ? lane - 8 * dd : lane;
    const double x0 = shfl_f64(u0, src), x1 = shfl_f64(u1, src);
    if (ss >= 0) {
      u0 = fma(p8a.x, x0, fma(p8a.y, x1, u0));
      u1 = fma(p8b.x, x0, fma(p8b.y, x1, u1));
    }
    if (lv < 2) {  // D^(8 TSUB 2^(lv+1)) = (D^(8 TSUB 2^lv))^2
      const f64x2 qa = f64x2{fma(p8a.x, p8a.x, p8a.y * p8b.x), fma(p8a.x, p8a.y, p8a.y * p8b.y)};
      const f64x2 qb = f64x2{fma(p8b.x, p8a.x, p8b.y * p8b.x), fma(p8b.x, p8a.y, p8b.y * p8b.y)};
      p8a = qa;
      p8b = qb;
    }
  }
  {
    const int ss = sg - 1;
    const int src = ss >= 0 ? lane - 8 : lane;
    const double x0 = shfl_f64(u0, src), x1 = shfl_f64(u1, src);
    u0 = ss >= 0 ? x0 : mi.x;
    u1 = ss >= 0 ? x1 : mi.y;
  }
  // (every lane stores: the idle lanes 6 and 7 of a segment both to the
  // row's padding slot 6 -- no exec masking per row, one address register)
  f64x2* const wr = reinterpret_cast<f64x2*>(rows + (8 * sg + 1) * kScanRow) + (kb < 6 ? kb : 6);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const double n0 = fma(d0a.x, u0, fma(d0a.y, u1, e[i].x));
    const double n1 = fma(d0b.x, u0, fma(d0b.y, u1, e[i].y));
    u0 = n0;
    u1 = n1;
    wr[i * (kScanRow / 2)] = f64x2{u0, u1};
  }
  static_assert(kScanRow == 14, "six blocks and one padding slot per scan row");
  // ---- 4. publish the tile's end state (segment 7's workers hold v_63); the
  // channel's last tile too, for the repair kernel (no flag: nobody waits)
  {
    const int64_t me = b * a.ntiles + tile;
    if (worker && sg == 7) {
      store_state(a.states + me * kD + 2 * kb, u0);
      store_state(a.states + me * kD + 2 * kb + 1, u1);
    }
    if constexpr (kRegCarry) {
      entry.c0 = u0;
      entry.c1 = u1;
    }
  }
  // The flag follows once these state stores are acknowledged; the y stores
  // below go out first, so that the wave does not sit in vmcnt(0) on the
  // stores' round trip (round 4): the wait counts the y stores as younger.
  const bool raise = !kRegCarry && tile + 1 < a.ntiles;
  auto raise_flag = [&] {
    if (lane == 8 * 7) store_flag(a.flags + b * a.ntiles + tile, 1u);
  };
  fence();
  double m[kD];
  {
    const double* src = lane == 0 ? park : rows + lane * kScanRow;
#pragma unroll
    for (int k = 0; k < kS; ++k) {
      const f64x2 t = *reinterpret_cast<const f64x2*>(src + 2 * k);
      m[2 * k] = t.x;
      m[2 * k + 1] = t.y;
    }
  }
  fence();

  // ---- 5. y out (unless the caller passed y = NULL), DF2 entry state
  // s = T m, pass 2, z out
  // (the buffer resources start at the tile's first output, so that the store
  // offsets are lane- and k-terms only; their size keeps the row-end checks)
  if (YST && a.y) {
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        a.y + b * a.ld_y + m0, 0, (int)((a.n_out - m0) * 4), 0x00020000);
    store_tile<TS>(lds, y, lane, ry);
    if (raise) {
      // every store but store_tile's TS / 4 (two halves of TS / 8) is done
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TS / 4) : "memory");
      raise_flag();
    }
  } else if (raise) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raise_flag();
  }
  pin(y);
  pass2_cascade<TS, REPAIR>(a, mt, y, m);
  const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(
      a.z + b * a.ld_y + m0, 0, (int)((a.n_out - m0) * 4), 0x00020000);
  int lane_z = lane;
  asm volatile("" : "+v"(lane_z));  // recompute the store offsets (no spill across pass 2)
  store_tile<TS>(lds, y, lane_z, rz);
}

// Repair kernels (k_chain_*_repair), launched after every single-pass kernel
// on its stream.  Each wave reads the last end state of 64 channels at a time
// (B * 8 bytes for the whole launch: a clean launch costs a few microseconds)
// and reruns every channel whose state is not finite (repair_channel).
// A channel's tiles run in order from its first tile with a non-finite end
// state: the tile before it is clean and its published end state is the entry
// state; later ones take this loop's own, through the hand-off protocol itself
// (the flag is raised here, consumed and cleared by tile_entry_state, and
// the flag a rerun tile raised is cleared after it).  A rerun of a tile whose
// window is clean gives the single-pass kernel's y and z bitwise, so every
// tile from the first non-finite end state on is rerun: which of them are
// wrong (a NaN through a zero tap of a neighbouring output, a delay output
// that skipped its window) is not recorded anywhere.
template <class BODY>
__device__ __forceinline__ void repair_channel(const TileArgs& a, int lane, int64_t b,
                                               BODY&& body) {
  const double* st = a.states + b * a.ntiles * kD + (kD - 1);
  uint32_t* fl = a.flags + b * a.ntiles;
  int64_t first = a.ntiles;
  for (int64_t t0 = 0; t0 < a.ntiles && first == a.ntiles; t0 += kWave) {
    const int64_t t = t0 + lane;
    const uint64_t bad =
        __builtin_amdgcn_ballot_w64(t < a.ntiles && !__builtin_isfinite(st[t * kD]));
    if (bad) first = t0 + __builtin_ctzll(bad);
  }
  for (int64_t tile = first; tile < a.ntiles; ++tile) {
    if (lane == 0 && tile > 0) store_flag(fl + tile - 1, 1u);  // states[tile - 1]: the entry
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    body(tile);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) store_flag(fl + tile, 0u);  // no flag left raised for the next call
  }
}

// The repair kernels' channel loop: wave `wave` of `waves` per workgroup.
template <class BODY>
__device__ __forceinline__ void repair_channels(const TileArgs& a, int wave, int waves,
                                                BODY&& body) {
  const int lane = lane_id();
  const int64_t stride = (int64_t)gridDim.x * waves * kWave;
  for (int64_t b0 = ((int64_t)blockIdx.x * waves + wave) * kWave; b0 < a.B; b0 += stride) {
    const int64_t b = b0 + lane;
    const double last = b < a.B ? a.states[(b * a.ntiles + a.ntiles - 1) * kD + (kD - 1)] : 0.0;
    uint64_t bad = __builtin_amdgcn_ballot_w64(!__builtin_isfinite(last));
    while (bad) {
      const int64_t bb = b0 + __builtin_ctzll(bad);
      bad &= bad - 1;
      repair_channel(a, lane, bb, [&](int64_t tile) { body(bb, tile); });
    }
  }
}

// One tile of the L3/M2 kernel (REPAIR: the rerun with the non-finite path).
template <class GEO, bool DLY, bool REPAIR>
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
  if (!REPAIR && tile > 0 && lane == 0) fl = load_flag(a.flags + b * a.ntiles + tile - 1);

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
  if (!REPAIR && tile > 0 && __builtin_amdgcn_readfirstlane(fl) == 1u) {
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
template <bool UP, bool REPAIR>
__device__ __forceinline__ void chain_gen_body(const TileArgs& a, const float* seq,
                                               const uint32_t* adv, float* win, int lane,
                                               int64_t b, int64_t tile) {
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
    tile_cascade<kGenTS>(a, mt, win, y, lane, b, tile, m0, 0);
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
template <int L, int M, bool T7, bool REPAIR>
__device__ __forceinline__ void chain_gct_body(const TileArgs& a, const float* seq, float* win,
                                               int lane, int64_t b, int64_t tile) {
  const int64_t qa = gen_window_start<L, M>(a, tile);
  gen_load_window(a, win, lane, b, qa);
  fence();
  gct_tile<L, M, T7, REPAIR>(a, seq, win, lane, b, tile, qa);
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
  int kind;  // 1: k_chain_tile<Geo3241>, 2: k_chain_gen, 3: k_chain_gct<160, 147>
  int64_t tsub, tile, ntiles;
  int win;   // kind 2: floats of a wave's x window
};

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
  if (S < 0 || S > kS || n_in < 1 || n_out < 1 || n_in % 4 || L < 1 || M < 1 || K < 1) return false;
  if (L == 1 && M == 1) return false;  // SRC bypass: the caller's cascade path
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
  const int64_t v[] = {4 /* table layout version */, tp.kind, tp.tsub, n_in, n_out, K, L, M, c, S,
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

}  // namespace

int64_t chain_tile_sub(int64_t n_in, int64_t n_out, int K, int L, int M, int64_t c, int S) {
  TilePlan tp;
  return tile_geometry(n_in, n_out, K, L, M, c, S, &tp) ? tp.tsub : 0;
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
  } else gen_sequences(ft.data(), K, L, M, c, tt);
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
  for (int r = 0; r < kD; ++r)
    for (int c = 0; c < kD; ++c) tt->Q[r][c] /= p.G;
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
  auto aligned = [](const void* p, int64_t ld) {
    return (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
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
  const int64_t groups = tp.kind == 1 ? B : ceil_div(B, (int64_t)kGenWaves);
  const int64_t rwaves = tp.kind == 1 ? 1 : kGenWaves;
  const unsigned rgrid =
      (unsigned)std::min<int64_t>(ceil_div(B, kWave * rwaves), kRepairGroups);
  if (tp.kind == 1) {
    // (No persistent variant: one measured 9 % slower at config 4 and 5 % at
    // config 3 than these chained tiles, profiles/r04_tilep_ab.txt.)
    {
      TraceScope trace("chain_tile", s);
      auto kern = dly ? k_chain_tile<Geo3241, true> : k_chain_tile<Geo3241, false>;
      hipLaunchKernelGGL(kern, dim3((unsigned)B, (unsigned)tp.ntiles), dim3(kWave), 0, s, a);
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
    const bool persistent = fits && res > 0 && groups >= res &&
                            groups * 8 >= rounds * res * 7 && variant != 2;
    {
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
    {
      TraceScope trace("chain_tile", s);
      hipLaunchKernelGGL(kern, dim3((unsigned)groups, (unsigned)tp.ntiles), dim3(kWave * kGenWaves), shm,
                         s, a);
    }
    TraceScope trace("chain_repair", s);
    hipLaunchKernelGGL(rep, dim3(rgrid), dim3(kWave * kGenWaves), shm, s, a);
  }
  DSP_LAUNCHED("k_chain_tile");
  return DSP_OK;
}

}  // namespace dsp
