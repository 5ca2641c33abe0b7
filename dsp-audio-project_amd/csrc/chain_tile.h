// Shared device code of the single-pass chain kernels (chain_tile.hip and
// chain_pp*.hip): tables, tile hand-off, pass 1, the carry scan, pass 2,
// the staged stores and the repair loop.  See chain_tile.hip's file comment
// for the decomposition and the hand-off protocol.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>

#include "cascade.h"

namespace dsp {


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

// Per-phase kernels (chain_pp.h): output slots (L' or 2 L' of them) and the
// floats of their tap rows.
constexpr int kPpSlots = 16;
constexpr int kPpTapFloats = 1024;

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
  // k_chain_pp (chain_pp.h, round 6): one row of tap pairs per output slot,
  // tpw[(slot * pp_np + p) * 2 + e] = h[2 p + e - s(slot)] of the slot's
  // branch, and the delay branch's centre tap.
  alignas(16) float tpw[kPpTapFloats];
  float pp_td;
  int32_t pp_np, pp_geo, pad4;
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
    } else if constexpr (TS != 48) {
      // any other TS (the per-phase kernels, chain_pp.h): row stride TS + 4,
      // the offset of g = 4 (lane + 64 k) computed per k
      static_assert(TS % 4 == 0, "staging rows of whole float4s");
      b[0] = lane;
    } else {
      const int a = (lane * 43) >> 9;  // lane div 12 (lane < 64)
      const int r = lane - 12 * a;
      b[0] = 4 * lane + 4 * a;
      b[1] = b[0] + 4 * ((r + 8) >> 4);   // + 4 [r >= 8]
      b[2] = b[0] + 4 * ((r + 12) >> 4);  // + 4 [r >= 4]
    }
  }
  __device__ __forceinline__ int at(int k) const {
    if constexpr (TS == 32) return b[0] + 256 * k;
    else if constexpr (TS != 48) {
      const int g = 4 * (b[0] + kWave * k);
      return g + 4 * (g / TS);
    } else return b[k % 3] + 276 * k + (k >= 3 ? 4 : 0);
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
  constexpr int NR = (NF4 + kWave - 1) / kWave;  // store rounds per half (the last may be partial)
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
    for (int k = 0; k < NR; ++k) {
      // output float g = 4 (lane + 64 k) sits in row r = g div TS at r RS + g
      // mod TS = g + 4 r (StageBase)
      const int g = 4 * (lane + kWave * k);
      // A partial last round (TS not a multiple of 8: the per-phase kernels)
      // stores from every lane, those past the half's outputs at an offset the
      // resource drops: no branch, so the y stores a counted hand-off wait
      // relies on (tile_cascade, vmcnt(TS / 4) <= 2 NR) are issued on every
      // path (tools/isa_count.py --check-handoff).
      const bool past = NF4 % kWave && k == NR - 1 && lane + kWave * k >= NF4;
      const float4 f = *reinterpret_cast<const float4*>(lds + sb.at(k));
      u32x4 d;
      d.x = __float_as_uint(f.x);
      d.y = __float_as_uint(f.y);
      d.z = __float_as_uint(f.z);
      d.w = __float_as_uint(f.w);
      __builtin_amdgcn_raw_buffer_store_b128(d, rs, past ? 0x7ffffff0 : (h * (kWave / 2) * TS + g) * 4,
                                             0, kStream);
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

// Pass 1 in float64 (the per-phase kernels, chain_pp.h): E' = sum_i G'[i] y[i]
// straight in block-diagonal coordinates, G'[i] = T^-1 A^(TS-1-i) B / gain
// (the tables' G; the 1 / gain as in Q), one float64 FMA chain per component,
// samples ascending.  12 float64 FMAs per sample instead of 6 v_pk_fma_f32 +
// the change of basis; no float32 rounding of the sums, which at the app's
// low output rates (6..35 kHz) took z 2.0-3.3e-6 from the two-launch chain.
template <int TS>
__device__ __forceinline__ void pass1_state_f64(tt_ptr mt, const float (&y)[TS], double (&v)[kD]) {
#pragma unroll
  for (int d = 0; d < kD; ++d) v[d] = 0.0;
#pragma unroll
  for (int i = 0; i < TS; ++i) {
    tt_ptr tq = mt;
    asm volatile("" : "+s"(tq));
    const double u = (double)y[i];
#pragma unroll
    for (int d = 0; d < kD; ++d) v[d] = fma(tq->G[i][d], u, v[d]);
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
template <int TS, bool P1F64 = false, class SUMS>
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
  } else if constexpr (P1F64) {
    // pass1_state_f64's sums in its order (bitwise the same E'), rolled
#pragma unroll
    for (int d = 0; d < kD; ++d) v[d] = 0.0;
#pragma unroll 1
    for (int i = 0; i < TS; ++i) {
      const double u = (double)get(i);
#pragma unroll
      for (int d = 0; d < kD; ++d) v[d] = fma(mt->G[i][d], u, v[d]);
    }
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
// The three-launch mode of small batches (round 6; chain_pp.h, the cascade
// alone): a chained hand-off costs ~2 us per tile, so a channel of many tiles
// waits ntiles x 2 us however few channels there are.  Instead, launch 1
// (AggEntry) runs every tile from a zero entry state and publishes only that
// end state -- the tile's aggregate -- in states[tile]; launch 2
// (k_tile_carry) scans the aggregates of each channel into the tiles' entry
// states, in place; launch 3 (GivenEntry) reruns every tile from its entry
// state and publishes its end state over it (for the repair kernel), no flag.
struct AggEntry {};
struct GivenEntry {};

template <int TS, bool YST = true, bool REPAIR = false, bool P1F64 = false, class ONNF,
          class ENTRY = ChainedEntry>
__device__ __forceinline__ void tile_cascade(const TileArgs& a, tt_ptr mt, float* lds,
                                             float (&y)[TS], int lane, int64_t b, int64_t tile,
                                             int64_t m0, ONNF&& on_nf, ENTRY&& entry = ENTRY{}) {
  constexpr bool kRegCarry = std::is_same_v<std::decay_t<ENTRY>, RegCarry>;
  constexpr bool kEarly = std::is_same_v<std::decay_t<ENTRY>, EarlyEntry>;
  constexpr bool kAgg = std::is_same_v<std::decay_t<ENTRY>, AggEntry>;
  constexpr bool kGiven = std::is_same_v<std::decay_t<ENTRY>, GivenEntry>;
  // ---- 2. pass 1: zero-state end state of the sub-chunk
  double v[kD];
  if constexpr (P1F64) pass1_state_f64<TS>(mt, y, v);
  else pass1_state<TS>(mt, y, v);
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
  if constexpr (kGiven) {
    // (launch 2 wrote the entry state over the aggregate)
    if (lane == 0) {
      const int64_t me = b * a.ntiles + tile;
#pragma unroll
      for (int k = 0; k < kS; ++k)
        *reinterpret_cast<f64x2*>(park + 2 * k) =
            *reinterpret_cast<const f64x2*>(a.states + me * kD + 2 * k);
    }
  } else if (kAgg || tile == 0) {
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
  if constexpr (kAgg) return;  // launch 1: the aggregate is all it computes
  const bool raise = !kRegCarry && !kGiven && tile + 1 < a.ntiles;
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

}  // namespace dsp
