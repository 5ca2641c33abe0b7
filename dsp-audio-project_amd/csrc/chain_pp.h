// Per-phase single-pass SRC -> biquad cascade kernels (round 6): the
// single-pass chain of chain_tile.hip for every SRC ratio the reference app
// offers -- L, M in 1..8 (/root/reference/app.py:149-150) at the default tap
// rule K = 40 max(L, M) + 1 (/root/reference/modules/dsp_core.py:158) -- and
// config 1's 2/1 at K = 127.  Same tile decomposition, hand-off, carry and
// pass 2 as k_chain_tile (chain_tile.h, tile_cascade); what changes is the SRC.
//
// Reduced ratio.  With g = gcd(L, M), L = g L', M = g M', c = g c1 + rho:
//   j = m M + c,  phi = j mod L = g ((m M' + c1) mod L') + rho,
//   q = j div L = (m M' + c1) div L',
// so the phase pattern is that of L'/M' and only the taps of the branches
// phi = g phi' + rho are used.  Lane l of a tile owns TS consecutive outputs,
// TS a multiple of L': every lane sees the same branch sequence, so output i
// of the lane's sub-chunk has a compile-time branch SLOT (i mod L', or i mod
// 2 L' when M' is odd: the window parity alternates then) and a compile-time
// window offset Qc(i) = i M' div L' from the lane's first input sample
// (lane stride LS = TS M' / L' inputs).  The run-time rest -- r0 = c1 mod L'
// (which branch and carry delta(i) in {0, 1} the slots get) and the window's
// float4 alignment A -- the host folds into each slot's tap row as a shift
// s = A + (Qc(i) mod 2) + delta(i): output i sums its row of NP tap pairs
// against the window pairs from E(i) = Qc(i) rounded down to even, all at
// compile-time register indices.  Rows are wave-uniform: the taps come
// through the scalar cache (TileTables::tpw), two per v_pk_fma_f32 whose
// halves keep the even- and odd-indexed x samples' partial sums -- the
// summation order of k_src_reg / k_src_generic (src_poly.hip), so y is
// bitwise the two-launch chain's.
//
// The cascade alone (ratio 1/1 at K = 1, chain_pp_list.h entry 0): the SRC
// bypass (dsp_core.py:144-145) as the one-tap SRC y = 1.0 x, every output a
// delay output, the lane windows back to back (LS = TS): x is read once and z
// written once, y (= x) never stored -- sistema_ecualizador (dsp_core.py:
// 216-254) in one pass instead of the two-pass cascade's x read twice.
//
// Delay branch (upsampling ratios, UC >= 0).  With wc = 1/L (dsp_core.py:155
// for L >= M) sinc(n / L) vanishes at every n = k L, so the branch of the
// centre tap -- slots i = 0 mod L' -- holds that tap alone once the library
// flushes the sinc-zero noise (common.h kTapFlushRel): those outputs are one
// multiply of the centre tap and one window sample at Qc(i) + UC, bitwise
// what the FMA chain gives (chain_tile.hip, DLY).  The host checks the rows
// (A = 0, every other tap of the slot zero) before it picks these kernels.
//
// Registers: the SRC runs in parts of NH outputs, each over blocks of PB tap
// pairs whose window slice (float4s from LDS) is loaded per block, next to
// y[TS] (tools/gen_chain_pp.py picks NH and PB for ~104 VGPRs; 4 waves per
// SIMD).  LDS: the tile's x window, padded by PAD floats per LS so that the
// lanes' ds_read_b128 (stride LS + PAD floats, an odd number of float4s)
// take distinct bank quads; the store staging and the scan rows reuse it.
#pragma once
#include "chain_tile.h"

// The instantiation list (tools/gen_chain_pp.py); -DPP_LIST='"file"' builds
// a variant library for A/B timing (tools/build_pp_variant.sh).
#ifndef PP_LIST
#define PP_LIST "chain_pp_list.h"
#endif

namespace dsp {

__host__ __device__ constexpr int pp_pad(int ls) { return (((ls + 4) / 4) % 2) ? 4 : 8; }

template <int LR_, int MR_, int TS_, int NP_, int UC_, int NH_, int PB_>
struct PpGeo {
  static constexpr int LR = LR_, MR = MR_, TS = TS_, NP = NP_, UC = UC_, NH = NH_, PB = PB_;
  static_assert(TS % LR == 0, "wave-uniform branches: TS a multiple of L'");
  static_assert(TS % 4 == 0 && TS <= 64, "whole float4 staging rows; pass-1 rows <= 32 pairs");
  static constexpr int LS = TS * MR / LR;  // input samples per lane
  static_assert((TS * MR) % LR == 0 && LS % 4 == 0, "lane windows on float4 boundaries");
  static constexpr int P = (MR % 2) ? 2 * LR : LR;  // output slots
  static_assert(P <= kPpSlots && P * NP * 2 <= kPpTapFloats, "tap rows");
  static_assert(PB == NP || PB % 2 == 0, "window blocks on float4 boundaries");
  static constexpr int TILE = kWave * TS;
  static constexpr int Qc(int i) { return i * MR / LR; }
  static constexpr int E(int i) { return Qc(i) & ~1; }
  static constexpr int slot(int i) { return i % P; }
  static constexpr bool dly(int i) { return UC >= 0 && i % LR == 0; }
  static constexpr int PAD = pp_pad(LS);
  static constexpr int LSP = LS + PAD;                          // lane stride in LDS
  static constexpr int W = E(TS - 1) + 2 * NP;                  // lane window (floats)
  static constexpr int NWIN = (LS * (kWave - 1) + W + 3) / 4 * 4;  // tile window
  static constexpr int xpos(int g) { return g + PAD * (g / LS); }   // padded LDS float
  static constexpr int XF = xpos(NWIN + 4) + 4;  // (+4: a part's last float4 may reach past W)
  static constexpr int SF = staging_floats(TS);
  // The one-tap SRC bypass (the cascade alone): lane windows back to back,
  // every window sample an output.  Its single-pass kernel stages the tile's
  // x through LDS in two halves of 32 lane windows (XH floats), so that its
  // LDS fits 4 waves per SIMD; the repair kernel keeps the whole window.
  static constexpr bool IDENT = LR == 1 && MR == 1 && NP == 1 && UC == 0;
  static_assert(!IDENT || (W == TS && LS == TS), "bypass windows back to back");
  static constexpr int XH = (kWave / 2) * LSP;
  static constexpr int LDSF0 = (IDENT ? XH : XF) > SF ? (IDENT ? XH : XF) : SF;
  static constexpr int LDSF = (LDSF0 > kScanFloats ? LDSF0 : kScanFloats) + 3 & ~3;
  static constexpr int LDSR0 = XF > SF ? XF : SF;  // repair kernel
  static constexpr int LDSR = (LDSR0 > kScanFloats ? LDSR0 : kScanFloats) + 3 & ~3;
};

// SRC outputs H0 .. H0+NH-1 of the lane's sub-chunk (the non-delay ones),
// from the lane's window at xw (padded LDS), tap pairs in blocks of PB.
template <class G, int H0, int NH>
__device__ __forceinline__ void pp_src_part(const float* xw, tt_ptr tt, float (&y)[G::TS]) {
  constexpr int H1 = H0 + NH <= G::TS ? H0 + NH : G::TS;
  constexpr int ND = [] {
    int n = 0;
    for (int i = H0; i < H1; ++i) n += G::dly(i) ? 0 : 1;
    return n;
  }();
  if constexpr (ND == 0) return;  // delay outputs only (pp_src did them)
  constexpr int NB = (G::NP + G::PB - 1) / G::PB;
  constexpr int V0 = G::E(H0) & ~3;                              // the part's first float4
  constexpr int NQ = (G::E(H1 - 1) + 2 * G::PB - V0 + 3) / 4;    // float4s per block
  f32x2 acc[H1 - H0];
#pragma unroll
  for (int i = 0; i < H1 - H0; ++i) acc[i] = f32x2{0.f, 0.f};
#pragma unroll
  for (int blk = 0; blk < NB; ++blk) {
    const int p0 = blk * G::PB;
    const int v0 = V0 + 2 * p0;  // a multiple of 4 (PB even, or one block)
    // (the last block loads only the float4s its pairs p < NP reach: never
    // past the window image)
    const int nq = (G::E(H1 - 1) + 2 * (G::NP - p0 < G::PB ? G::NP - p0 : G::PB) - V0 + 3) / 4;
    f32x2 w[2 * NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      if (k >= nq) break;
      const f32x4 f = *reinterpret_cast<const f32x4*>(xw + G::xpos(v0 + 4 * k));
      w[2 * k] = f32x2{f.x, f.y};
      w[2 * k + 1] = f32x2{f.z, f.w};
    }
#pragma unroll
    for (int pp = 0; pp < G::PB; ++pp) {
      const int p = p0 + pp;
      if (p >= G::NP) break;
      // each pair's taps scalar-loaded right before its FMAs (an opaque table
      // pointer per pair: the compiler does not hoist every row into SGPRs)
      tt_ptr tq = tt;
      asm volatile("" : "+s"(tq));
      f32x2 t[G::P];
#pragma unroll
      for (int sl = 0; sl < G::P; ++sl)
        t[sl] = f32x2{tq->tpw[(sl * G::NP + p) * 2], tq->tpw[(sl * G::NP + p) * 2 + 1]};
#pragma unroll
      for (int i = H0; i < H1; ++i) {
        if (G::dly(i)) continue;
        acc[i - H0] = __builtin_elementwise_fma(t[G::slot(i)], w[(G::E(i) - v0) / 2 + p], acc[i - H0]);
      }
    }
    pin(acc);
  }
#pragma unroll
  for (int i = H0; i < H1; ++i)
    if (!G::dly(i)) y[i] = acc[i - H0].x + acc[i - H0].y;
}

template <class G, int H0>
__device__ __forceinline__ void pp_src_parts(const float* xw, tt_ptr tt, float (&y)[G::TS]) {
  if constexpr (H0 < G::TS) {
    pp_src_part<G, H0, G::NH>(xw, tt, y);
    pin(y);
    pp_src_parts<G, H0 + G::NH>(xw, tt, y);
  }
}

// The lane's TS outputs: delay outputs first (one LDS read and one multiply
// each), then the FMA parts.
template <class G>
__device__ __forceinline__ void pp_src(const float* xw, tt_ptr tt, float (&y)[G::TS]) {
  if constexpr (G::UC >= 0) {
    tt_ptr tq = tt;
    asm volatile("" : "+s"(tq));
    const float td = tq->pp_td;
#pragma unroll
    for (int i = 0; i < G::TS; i += G::LR) y[i] = td * xw[G::xpos(G::Qc(i) + G::UC)];
    if constexpr (G::LR == 1 && G::W > G::TS) {
      // every output a delay output (L = M): no FMA meets the rest of the
      // window, so an inf or NaN there would not reach the tile's end state
      // and the repair kernel.  (W == TS: the one-tap SRC bypass, whose
      // outputs are the whole window, needs no flag.)  Flag it (fma(x, 0, acc) is NaN exactly for a
      // non-finite x): y[0] becomes NaN, the repair reruns the channel and
      // recomputes every output with the reference's semantics.
      f32x2 acc = {0.f, 0.f};
#pragma unroll
      for (int v = 0; v < G::W; v += 4) {
        const f32x4 f = *reinterpret_cast<const f32x4*>(xw + G::xpos(v));
        acc = __builtin_elementwise_fma(f32x2{f.x, f.y}, f32x2{0.f, 0.f}, acc);
        acc = __builtin_elementwise_fma(f32x2{f.z, f.w}, f32x2{0.f, 0.f}, acc);
      }
      if (!__builtin_isfinite(acc.x + acc.y)) y[0] = __builtin_nanf("");
    }
  }
  pp_src_parts<G, 0>(xw, tt, y);
}

// Pass 1 of the per-phase kernels: float32 sums in input-normal coordinates
// as k_chain_tile's (false), or float64 in block-diagonal ones
// (pass1_state_f64: measured no closer to the two-launch chain at the app's
// low output rates -- the float32 rounding of y dominates there -- and 2/1
// no faster by it: 1.236 vs 1.228 ms at 4096 channels).
constexpr bool kPpP1F64 = false;

// One tile (REPAIR: the rerun with the non-finite path): the x window, the
// SRC, then tile_cascade as k_chain_tile (early hand-off included).
// MODE: 0 the chained hand-off, 1 / 2 launch 1 / 3 of the three-launch mode
// (chain_tile.h, AggEntry / GivenEntry).
template <class G, bool REPAIR, int MODE = 0>
__device__ __forceinline__ void chain_pp_body(const TileArgs& a, float* lds, int lane, int64_t b,
                                              int64_t tile) {
  constexpr int TS = G::TS;
  const int64_t m0 = tile * G::TILE;
  const tt_ptr mt = (tt_ptr)a.tt;
  uint32_t fl = 0;
  if (!REPAIR && MODE == 0 && tile > 0 && lane == 0)
    fl = load_flag(a.flags + b * a.ntiles + tile - 1);
  // ---- x window of the tile -> padded LDS image (zeros outside [0, n_in));
  // its first sample xa = tile * 64 LS + cq is a multiple of 4 (the host's
  // alignment A went into the tap rows)
  const int64_t xa = tile * (int64_t)(kWave * G::LS) + a.cq;
  float y[TS];
  if constexpr (G::IDENT && !REPAIR) {
    // the cascade alone: all 12 float4 loads of the lane in flight at once
    // (float4 f = lane + 64 k of the tile's 64 TS samples, coalesced), then
    // the two halves through LDS, each read back by its 32 lanes as their
    // y = td x (td = 1.0 for the bypass)
    static_assert(TS == 48 && G::XH <= G::LDSF, "two halves of 32 x 48 samples");
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.x) + b * a.ld_x, 0, (int)(a.n_in * 4), 0x00020000);
    constexpr int NF = kWave * TS / 4 / kWave;  // float4s per lane: 12
    f32x4 v[NF];
    const int off0 = (int)(xa * 4) + 16 * lane;
#pragma unroll
    for (int k = 0; k < NF; ++k)
      v[k] = __builtin_amdgcn_raw_buffer_load_b128(rx, off0 + 1024 * k, 0, kStream);
    tt_ptr tq = mt;
    asm volatile("" : "+s"(tq));
    const float td = tq->pp_td;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int k = 0; k < NF / 2; ++k)
        *reinterpret_cast<f32x4*>(lds + G::xpos(4 * (lane + kWave * k))) = v[h * (NF / 2) + k];
      fence();
      if ((lane >> 5) == h) {
        const float* xw = lds + G::LSP * (lane & 31);
#pragma unroll
        for (int j = 0; j < TS / 4; ++j) {
          const f32x4 f = *reinterpret_cast<const f32x4*>(xw + 4 * j);
          y[4 * j] = td * f.x;
          y[4 * j + 1] = td * f.y;
          y[4 * j + 2] = td * f.z;
          y[4 * j + 3] = td * f.w;
        }
      }
      fence();
    }
  } else {
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.x) + b * a.ld_x, 0, (int)(a.n_in * 4), 0x00020000);
    constexpr int NF = G::NWIN / 4;
    const int off0 = (int)(xa * 4) + 16 * lane;
#pragma unroll
    for (int k = 0; k < (NF + kWave - 1) / kWave; ++k) {
      const int f = lane + kWave * k;
      if ((k + 1) * kWave <= NF || f < NF) {
        // ("negative" offsets of tile 0 are >= 2^31 as unsigned: zeros)
        const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rx, off0 + 1024 * k, 0, kStream);
        *reinterpret_cast<f32x4*>(lds + G::xpos(4 * f)) = v;
      }
    }
    fence();  // one wave: its LDS operations execute in order
  }
  EarlyEntry early{false, reinterpret_cast<const double*>(lds + G::LDSF)};
  if (!REPAIR && MODE == 0 && tile > 0 && __builtin_amdgcn_readfirstlane(fl) == 1u) {
    early.early = true;
    if (lane < 2 * kD) {
      const int64_t prev = b * a.ntiles + tile - 1;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(reinterpret_cast<const uint32_t*>(
                                                               a.states + prev * kD) + lane),
          (__attribute__((address_space(3))) void*)(lds + G::LDSF), 4, 0, kSc1);
    }
  }
  // ---- 1. SRC
  if constexpr (!G::IDENT || REPAIR) pp_src<G>(lds + G::LSP * lane, mt, y);
  pin(y);
  if constexpr (REPAIR) {
    auto fix = [&](float (&yy)[TS], double (&v)[kD]) {
      const float thr = mt->flush_thr;
      const int64_t j0 = (m0 + (int64_t)TS * lane) * a.M + a.c;
      fix_outputs<TS, kPpP1F64>(a, mt, b, m0 + TS * lane, yy, v, [&](int i, float& nf, float& fin) {
        const int64_t j = j0 + (int64_t)i * a.M, q = j / a.L;
        const int base = (int)(q - xa);  // x[q] in the window; xa is a multiple of 4
        window_sums(a.taps, a.K, a.L, (int)(j - q * a.L), thr, base,
                    [&](int t) { return lds[G::xpos(base - t)]; }, nf, fin);
      });
    };
    tile_cascade<TS, true, true, kPpP1F64>(a, mt, lds, y, lane, b, tile, m0, fix);
  } else {
    if constexpr (MODE == 1)
      tile_cascade<TS, true, false, kPpP1F64>(a, mt, lds, y, lane, b, tile, m0, 0, AggEntry{});
    else if constexpr (MODE == 2)
      tile_cascade<TS, true, false, kPpP1F64>(a, mt, lds, y, lane, b, tile, m0, 0, GivenEntry{});
    else
      tile_cascade<TS, true, false, kPpP1F64>(a, mt, lds, y, lane, b, tile, m0, 0, early);
  }
}

template <class G>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(4))) void k_chain_pp(
    TileArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[G::LDSF + 2 * kD];  // + the early slot
  chain_pp_body<G, false>(a, lds, threadIdx.x, blockIdx.x, blockIdx.y);
}

// Launches 1 and 3 of the three-launch mode (chain_tile.h, AggEntry).
template <class G, int MODE>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(4))) void k_chain_pp3(
    TileArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[G::LDSF];
  chain_pp_body<G, false, MODE>(a, lds, threadIdx.x, blockIdx.x, blockIdx.y);
}

template <class G>
__global__ __launch_bounds__(kWave) void k_chain_pp_repair(TileArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[G::LDSR + 2 * kD];
  repair_channels(a, 0, 1, [&](int64_t b, int64_t tile) {
    chain_pp_body<G, true>(a, lds, (int)threadIdx.x, b, tile);
  });
}

// Host: the geometry an instantiation serves (chain_pp_list.h rows).
struct PpEntry {
  int LR, MR, TS, NP, UC, NH, PB;
};

// Launch 2 of the three-launch mode (chain_tile.hip): the aggregates in
// states[] scanned into the tiles' entry states, per channel.
void launch_tile_carry(const TileArgs& a, int tile_len, hipStream_t s);

// Launches k_chain_pp<G> (three: the three-launch mode instead) and its
// repair kernel on s (the caller checked the geometry, tables
// and workspace: chain_tile.hip launch_chain_tile).
template <class G>
int pp_launch(const TileArgs& a, unsigned rgrid, bool three, hipStream_t s) {
  const dim3 grid((unsigned)a.B, (unsigned)a.ntiles);
  if (three) {
    {
      TraceScope trace("chain_tile_agg", s);
      hipLaunchKernelGGL((k_chain_pp3<G, 1>), grid, dim3(kWave), 0, s, a);
    }
    launch_tile_carry(a, G::TS, s);
    TraceScope trace("chain_tile", s);
    hipLaunchKernelGGL((k_chain_pp3<G, 2>), grid, dim3(kWave), 0, s, a);
  } else {
    TraceScope trace("chain_tile", s);
    hipLaunchKernelGGL(k_chain_pp<G>, grid, dim3(kWave), 0, s, a);
  }
  TraceScope trace("chain_repair", s);
  hipLaunchKernelGGL(k_chain_pp_repair<G>, dim3(rgrid), dim3(kWave), 0, s, a);
  DSP_LAUNCHED("k_chain_pp");
  return DSP_OK;
}

// One of the translation units chain_pp_<n>.hip: launches the entry `e`
// if that unit instantiates it, else kNotFused.
constexpr int kPpUnits = 4;
int launch_chain_pp_0(const PpEntry& e, const TileArgs& a, unsigned rgrid, bool three,
                       hipStream_t s);
int launch_chain_pp_1(const PpEntry& e, const TileArgs& a, unsigned rgrid, bool three,
                       hipStream_t s);
int launch_chain_pp_2(const PpEntry& e, const TileArgs& a, unsigned rgrid, bool three,
                       hipStream_t s);
int launch_chain_pp_3(const PpEntry& e, const TileArgs& a, unsigned rgrid, bool three,
                       hipStream_t s);

}  // namespace dsp
