// Biquad cascade (DF2T) for gfx950, float64 arithmetic, float32 I/O.
//
// Replaces reference modules/dsp_core.py:233-254: the serial loop of
// aplicar_ecuacion_diferencias (= scipy.signal.lfilter(b, a, x), :205-214) over
// the EQ bands followed by np.clip(y, -1, 1) (:254).  lfilter realises each
// biquad in direct form II transposed with zero initial state.  The kernels
// realise the same transfer functions in direct form II with the b0 gains
// pulled out (every b0 != 0, as for every EQ band):
//     u *= G = prod b0;  per stage:  w = u - a1 w1 - a2 w2
//                                    v = w + (b1/b0) w1 + (b2/b0) w2
// i.e. 4 fp64 FMAs per stage instead of DF2T's 4 FMAs + 1 multiply (25 vs 30
// per sample for the 6-band EQ); with some b0 == 0 the stage keeps its gain
// (v = b0 w + b1 w1 + b2 w2, NORM = false).  Both are exact rearrangements of
// the same recursion; in float64 they differ from lfilter's DF2T by rounding
// only (~1e-12 here against the 1e-5 tolerance).
// Float64 state and coefficients are mandatory: the 40 Hz band has poles at
// |r| = 0.99926 and a float32 recursion drifts by ~1e-3.
//
// Parallelism.  The recursion is serial in time and one lane per channel would
// leave the chip ~16x under-filled at 4096 channels, and fp64 FMAs need >= 4
// waves per SIMD to approach their issue rate (tools/ubench_fp64.hip).  The
// S-stage cascade is a D = 2S state linear system X' = A X + B u, so each
// channel's time axis is cut into C chunks of T samples and the exact initial
// state of every chunk is recovered by a carry scan:
//   pass 1: chunk end state from zero state, E_c = sum_n A^(T-1-n) B u[n]
//           - either by running the cascade (~30 fp64 ops per sample), or
//           - with the caller's state-response table G[t] = A^(T-1-t) B as a
//             2S-FMA-per-sample dot product (no recurrence, no dependency chain),
//           - or (chain) with G composed with the SRC taps, over the SRC input;
//   scan:   S_0 = 0, S_{c+1} = A^T S_c + E_c  (A^T is computed on the host);
//   pass 2: rerun every chunk from S_c, clip, store.
// With C <= 256 and S <= 8 all three run in ONE kernel (k_iir_wave).  With
// C <= 64 one wavefront owns one channel, lane c = chunk c, so tile staging, the
// carry scan and both passes are wave-private -- no workgroup barrier anywhere,
// and each wave streams independently of the others on its SIMD; up to 256
// chunks use four such waves per channel and a block-wide scan.  Otherwise the general
// path runs pass 1, a carry kernel and pass 2 as separate launches.  The
// chunking depends only on the caller's chunk_len, never on B, so a row's
// result is bitwise identical however the batch is sized or sharded.
//
// Memory.  Lanes are (channel, chunk) rows.  An NR-row x 32-sample fp32 tile is
// loaded with coalesced 128-byte row segments into LDS (row stride 33 floats:
// conflict-free per-lane column reads); the next tile's global loads are issued
// into registers before the current tile is computed, so HBM latency hides
// under the fp64 work.  Pass 2 writes its outputs back into the tile and stores
// it with the same coalesced pattern.
#include <climits>
#include <cmath>
#include <vector>

#include "cascade.h"

namespace dsp {
namespace {

struct ScanParams {
  double P[16 * 16];  // A^T, row-major D x D, D = 2S <= 16
};

constexpr int kNT = 256;       // lanes (rows) per block, general path
constexpr int kTS = 32;        // samples per tile step (chunk_len granule)
constexpr int kRow = kTS + 1;  // LDS row stride in floats
constexpr int kLoads = kTS / 4;  // float4 loads per thread per tile (one row per thread)
constexpr int kCBMax = 4 * kWave;  // max chunks per channel in the fused kernel
// Row descriptors live in LDS: global offset of the row's first sample for
// input and output, and the valid sample range [lo, len) of the row.
struct Rows {
  int64_t* in;
  int64_t* out;
  int* len;
  int* lo;
};

// Tile hand-off between the NR threads that share a tile.  NR == 64 (one
// wave): LDS instructions of a wave execute in program order, so a compiler
// fence suffices.  NR > 64: a workgroup barrier that waits only for LDS
// traffic -- __syncthreads() would also wait for vmcnt(0) and drain the next
// tile's prefetched loads and the previous tile's stores at every barrier.
template <int NR>
__device__ __forceinline__ void tile_sync() {
  if constexpr (NR == kWave) {
    asm volatile("" ::: "memory");
  } else {
    lds_barrier();
  }
}

// Issues this thread's kLoads float4 loads of tile [t0, t0+32) into registers
// (8 threads per row, 128 contiguous bytes).  tid is the thread's index among
// the NR threads sharing the tile.
// VEC (rows 16-byte aligned, ld % 4 == 0, lo % 4 == 0): branch-free -- every
// vector with at least one valid sample is loaded whole (ld % 4 == 0 and
// ld >= n keep the over-read inside the row pitch), others load a dummy vector
// at x; masking is deferred to tile_put so no wait lands between the loads and
// their use.  !VEC: guarded scalar loads (slow path for odd pitches).
template <int NR, bool VEC>
__device__ __forceinline__ void fetch(float4 (&v)[kLoads], const float* __restrict__ x,
                                      const Rows& rows, int t0, int tid) {
  const int c4 = (tid & 7) * 4;
#pragma unroll
  for (int i = 0; i < kLoads; ++i) {
    const int r = i * (NR / 8) + (tid >> 3);
    const int len = rows.len[r];
    const int t = t0 + c4;
    if constexpr (VEC) {
      const float* src = (t < len && t >= rows.lo[r]) ? x + rows.in[r] + t : x;
      v[i] = *reinterpret_cast<const float4*>(src);
    } else {
      const int lo = rows.lo[r];
      const float* src = x + rows.in[r] + t;
      v[i].x = (t + 0 < len && t + 0 >= lo) ? src[0] : 0.f;
      v[i].y = (t + 1 < len && t + 1 >= lo) ? src[1] : 0.f;
      v[i].z = (t + 2 < len && t + 2 >= lo) ? src[2] : 0.f;
      v[i].w = (t + 3 < len && t + 3 >= lo) ? src[3] : 0.f;
    }
  }
}

// Writes the fetched tile into LDS; MASK: zeroes samples outside each row's
// range (one unsigned compare per sample: t - lo < len - lo).
template <int NR, bool MASK>
__device__ __forceinline__ void tile_put(float* tile, const float4 (&v)[kLoads],
                                         const Rows& rows, int t0, int tid) {
  const int c4 = (tid & 7) * 4;
#pragma unroll
  for (int i = 0; i < kLoads; ++i) {
    const int r = i * (NR / 8) + (tid >> 3);
    float* d = tile + r * kRow + c4;
    if constexpr (MASK) {
      const int lo = rows.lo[r];
      const int len = rows.len[r];
      const uint32_t a = (uint32_t)(t0 + c4 - lo), w = len > lo ? (uint32_t)(len - lo) : 0u;
      d[0] = a + 0 < w ? v[i].x : 0.f;
      d[1] = a + 1 < w ? v[i].y : 0.f;
      d[2] = a + 2 < w ? v[i].z : 0.f;
      d[3] = a + 3 < w ? v[i].w : 0.f;
    } else {
      d[0] = v[i].x;
      d[1] = v[i].y;
      d[2] = v[i].z;
      d[3] = v[i].w;
    }
  }
}

// Stores this thread's kLoads vectors of the tile.  SM (store mode):
//   0: guarded float4 / scalar global stores (any pitch; general path);
//   1: one raw-buffer float4 store per vector, offset pushed out of range when
//      the vector is past the row's end -- branch-free, so the compiler can
//      count vmcnt exactly and the next tile's wait never drains these stores;
//   2: like 1 with four dword stores per vector (rows whose length is not a
//      multiple of 4 end in a partial vector).
// Modes 1-2 address y relative to the buffer resource's base (rows.out).
constexpr uint32_t kOob = 0x80000000u;  // > any buffer span (checked on host)

template <int NR, int SM>
__device__ __forceinline__ void tile_store(float* __restrict__ y, __amdgpu_buffer_rsrc_t rsrc,
                                           const float* tile, const Rows& rows, int t0,
                                           int tid) {
  const int c4 = (tid & 7) * 4;
#pragma unroll
  for (int i = 0; i < kLoads; ++i) {
    const int r = i * (NR / 8) + (tid >> 3);
    const int len = rows.len[r];
    const int t = t0 + c4;
    const float* s = tile + r * kRow + c4;
    if constexpr (SM == 0) {
      float* dst = y + rows.out[r] + t;
      if (t + 3 < len) {
        *reinterpret_cast<float4*>(dst) = make_float4(s[0], s[1], s[2], s[3]);
      } else {
        if (t + 0 < len) dst[0] = s[0];
        if (t + 1 < len) dst[1] = s[1];
        if (t + 2 < len) dst[2] = s[2];
        if (t + 3 < len) dst[3] = s[3];
      }
    } else if constexpr (SM == 1) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      u32x4 d;
      d.x = __float_as_uint(s[0]);
      d.y = __float_as_uint(s[1]);
      d.z = __float_as_uint(s[2]);
      d.w = __float_as_uint(s[3]);
      const uint32_t off = (t < len) ? (uint32_t)((rows.out[r] + t) * 4) : kOob;
      __builtin_amdgcn_raw_buffer_store_b128(d, rsrc, (int)off, 0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t off = (t + e < len) ? (uint32_t)((rows.out[r] + t + e) * 4) : kOob;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s[e]), rsrc, (int)off, 0, 0);
      }
    }
  }
}

// Affine row addressing for the one-channel-per-wave kernel (VM > 0): row r of
// a pass starts at byte r*stride*4 + start*4 of one channel's row, so vector i
// of a thread sits at base + i*step + t0*4 with base/step fixed for the pass.
// Loads and stores go through raw buffers spanning that channel's row only:
// offsets past the end (or "negative", i.e. >= 2^31) read zeros and drop
// stores in hardware, so neither needs a per-vector guard or a row descriptor.
struct AffIO {
  __amdgpu_buffer_rsrc_t in;
  int in_base, in_step;    // bytes
  int out_base, out_step;  // bytes, into the y buffer resource
};

__device__ __forceinline__ AffIO aff_rows(__amdgpu_buffer_rsrc_t in, int64_t in_stride,
                                          int64_t in_start, int64_t out_stride, int first_row,
                                          int tid) {
  const int r = first_row + (tid >> 3), c4 = (tid & 7) * 4;
  AffIO io;
  io.in = in;
  io.in_base = (int)(((int64_t)r * in_stride + in_start + c4) * 4);
  io.in_step = (int)(in_stride * 4 * (kWave / 8));
  io.out_base = (int)(((int64_t)r * out_stride + c4) * 4);
  io.out_step = (int)(out_stride * 4 * (kWave / 8));
  return io;
}

__device__ __forceinline__ void fetch_aff(float4 (&v)[kLoads], const AffIO& io, int t0) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int i = 0; i < kLoads; ++i) {
    const f32x4 a = __builtin_amdgcn_raw_buffer_load_b128(io.in, io.in_base + i * io.in_step + t0 * 4,
                                                          0, 0);
    v[i] = make_float4(a.x, a.y, a.z, a.w);
  }
}

template <int SM>
__device__ __forceinline__ void store_aff(__amdgpu_buffer_rsrc_t rsrc, const float* tile,
                                          const AffIO& io, int t0, int tid) {
  const int c4 = (tid & 7) * 4;
#pragma unroll
  for (int i = 0; i < kLoads; ++i) {
    const int r = i * (kWave / 8) + (tid >> 3);
    const float* s = tile + r * kRow + c4;
    const int off = io.out_base + i * io.out_step + t0 * 4;
    if constexpr (SM == 1) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      u32x4 d;
      d.x = __float_as_uint(s[0]);
      d.y = __float_as_uint(s[1]);
      d.z = __float_as_uint(s[2]);
      d.w = __float_as_uint(s[3]);
      __builtin_amdgcn_raw_buffer_store_b128(d, rsrc, off, 0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s[e]), rsrc, off + 4 * e, 0, 0);
    }
  }
}

enum PassMode { kStateCascade = 0, kStateTable = 1, kApply = 2 };

// One pass over every row of the NR-row group, tile by tile, with the next
// tile's loads in flight during the current tile's arithmetic.  Samples outside
// a row's range are zeros; their outputs are never stored.  Starts with a
// hand-off (fetch reads other threads' row descriptors) and ends with one.
template <int S, int MODE, int NR, int VM, bool VIN, bool NORM, bool AFF = false>
__device__ __forceinline__ void run_pass(const float* __restrict__ x, float* __restrict__ y,
                                         __amdgpu_buffer_rsrc_t rsrc, float* tile,
                                         const Rows& rows, const AffIO& io, int64_t T, int tid,
                                         double (&s1)[S > 0 ? S : 1],
                                         double (&s2)[S > 0 ? S : 1],
                                         double (&e)[S > 0 ? 2 * S : 1], const SosParams& p,
                                         const double* __restrict__ G, int clip) {
  constexpr int D = 2 * S;
  float* my = tile + tid * kRow;
  float4 v[kLoads];
  tile_sync<NR>();  // every thread's row descriptors are written
  if constexpr (AFF) fetch_aff(v, io, 0);
  else fetch<NR, VIN>(v, x, rows, 0, tid);
  // Tiles in [span_lo, span_hi) lie inside the range of every row of the wave
  // that has one and are put unmasked (a row without samples is a chunk whose
  // state is never used).  Pass 2 never masks: outputs past a row's end are
  // not stored.
  int span_lo = 0, span_hi = MODE == kApply ? INT_MAX : 0;
  if constexpr (NR == kWave && MODE != kApply) {
    const int len = rows.len[tid], lo = rows.lo[tid];
    int a = len > 0 ? lo : 0, z = len > 0 ? len : INT_MAX;
#pragma unroll
    for (int m = 1; m < kWave; m <<= 1) {
      a = max(a, __shfl_xor(a, m));
      z = min(z, __shfl_xor(z, m));
    }
    span_lo = __builtin_amdgcn_readfirstlane(a);
    span_hi = __builtin_amdgcn_readfirstlane(z);
  }
  const float clo = clip ? -1.f : -INFINITY, chi = clip ? 1.f : INFINITY;
  for (int t0 = 0; t0 < (int)T; t0 += kTS) {
    tile_sync<NR>();  // readers of the previous tile are done
    if (t0 >= span_lo && t0 + kTS <= span_hi)
      tile_put<NR, false>(tile, v, rows, t0, tid);
    else
      tile_put<NR, true>(tile, v, rows, t0, tid);
    tile_sync<NR>();
    if (t0 + kTS < (int)T) {
      if constexpr (AFF) fetch_aff(v, io, t0 + kTS);
      else fetch<NR, VIN>(v, x, rows, t0 + kTS, tid);
    }
    if constexpr (MODE == kStateTable) {
      const double* g = G + t0 * D;
#pragma unroll 4
      for (int j = 0; j < kTS; ++j) {
        const double u = (double)my[j];
#pragma unroll
        for (int i = 0; i < D; ++i) e[i] = fma(g[j * D + i], u, e[i]);
      }
    } else {
#pragma unroll 8
      for (int j = 0; j < kTS; ++j) {
        const float out = (float)cascade_step<S, NORM>((double)my[j], s1, s2, p);
        if constexpr (MODE == kApply) my[j] = clip_f32(out, clo, chi);
      }
    }
    if constexpr (MODE == kApply) {
      tile_sync<NR>();
      if constexpr (AFF) store_aff<VM>(rsrc, tile, io, t0, tid);
      else tile_store<NR, VM>(y, rsrc, tile, rows, t0, tid);
    }
  }
  tile_sync<NR>();
}

// ---------------------------------------------------------------------------
// Fused single-launch cascade: pass 1 + carry scan + pass 2, one wavefront per
// channel, lane c = chunk c (C <= 64 chunks of T samples).
// ---------------------------------------------------------------------------
// P1 (pass-1 mode): 0 = cascade run over the chunk, 1 = state-response table
// G[T][2S] over the chunk, 2 = state-response table projected onto the SRC
// input (chain only): when x = SRC(xs) the end state of chunk c is
//     E_c = sum_j Gx[j] xs[c*XS.shift + XS.q0 + j],  j < XS.rows,
// with Gx = G composed with the polyphase taps on the host in float64
// (dspcore/design.py:xstate_table).  Pass 1 then reads the SRC input (2/3 of
// the bytes at L/M = 3/2) and costs 2S*M/L FMAs per output sample instead of
// 2S, and the chunk states are those of the exact float64 SRC output.
struct XState {
  const float* xs;  // SRC input rows [B][ld]
  int64_t ld, n, shift, q0, rows;
  int64_t span;  // rows [0, span) meet a tap of the chunk (Gx is zero beyond)
};

// Per-wave LDS: the 64 x 33-float tile, reused as the 64 x D-double scan.
constexpr int kWaveTileFloats = kWave * kRow;

// W waves per channel (chunk c = 64*wave + lane, C <= 64*W).  W == 1: the
// scan is wave-synchronous and the kernel has no workgroup barrier.  W > 1
// (small batches: more chunks so that B*W waves still fill the chip): four
// barriers around a block-wide serial scan run by wave 0.
template <int W>
__device__ __forceinline__ void block_sync() {
  if constexpr (W == 1) asm volatile("" ::: "memory");
  else __syncthreads();
}

// Carry scan over the C chunks of one channel.  Slot c of `scan` ([C][2S]
// doubles in LDS) receives E_c; step cc overwrites slot cc with
// S_{cc+1} = P S_cc + E_cc (S_cc sits in slot cc-1), so chunk c >= 1 finds its
// initial state in slot c-1.  Lanes 0..D-1 of wave 0 each own one state
// component; a wave's LDS instructions execute in order.  c = thread index in
// the block (chunk); leaves chunk c's initial state in s1/s2.
template <int S, int W>
__device__ __forceinline__ void carry_scan(double* scan, const double (&e)[2 * S],
                                           double (&s1)[S], double (&s2)[S],
                                           const ScanParams& sp, int c, int C) {
  constexpr int D = 2 * S;
#pragma unroll
  for (int i = 0; i < D; ++i) scan[c * D + i] = e[i];
  const bool row_lane = c < D;
  double prow[D];
  if (row_lane) {
#pragma unroll
    for (int j = 0; j < D; ++j) prow[j] = sp.P[c * D + j];
  }
  block_sync<W>();
  if (c < kWave) {
    for (int cc = 0; cc + 1 < C; ++cc) {
      if (row_lane) {
        double acc = scan[cc * D + c];
        if (cc > 0) {
#pragma unroll
          for (int j = 0; j < D; ++j) acc = fma(prow[j], scan[(cc - 1) * D + j], acc);
        }
        asm volatile("" ::: "memory");  // all reads of S_cc precede the write
        scan[cc * D + c] = acc;
      }
      asm volatile("" ::: "memory");
    }
  }
  block_sync<W>();
  // Branch-free (a divergent branch here made the compiler select through a
  // scratch slot, whose reload then forced vmcnt(0) waits inside pass 2).
  const int src = c > 0 ? c - 1 : 0;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const double a1 = scan[src * D + 2 * k], a2 = scan[src * D + 2 * k + 1];
    s1[k] = c > 0 ? a1 : 0.0;
    s2[k] = c > 0 ? a2 : 0.0;
  }
  block_sync<W>();  // W > 1: states read before the tiles are reused
}

template <int S, int P1, int VM, bool NORM, int W>
__global__ __launch_bounds__(kWave * W) void k_iir_wave(
    const float* __restrict__ x, float* __restrict__ y, int64_t B, int64_t n,
    int64_t ld_x, int64_t ld_y, SosParams p, ScanParams sp,
    const double* __restrict__ G, int64_t T, int C, int clip, XState XS) {
  constexpr int D = 2 * S;
  static_assert(kWave * D * 2 <= kWaveTileFloats, "scan must fit in the tiles");
  __shared__ __attribute__((aligned(16))) float tiles[W * kWaveTileFloats];
  __shared__ int64_t s_in[kWave * W], s_out[kWave * W];
  __shared__ int s_len[kWave * W], s_lo[kWave * W];
  double* scan = reinterpret_cast<double*>(tiles);

  const int c = threadIdx.x;  // chunk
  const int lane = c & (kWave - 1), wv = c / kWave;
  float* tile = tiles + wv * kWaveTileFloats;
  const int64_t b = blockIdx.x;
  const bool live = c < C;
  const int64_t t_begin = (int64_t)c * T;
  // Pass-2 row descriptors (the x-state pass 1 reads other rows first).
  const int64_t in2 = live ? b * ld_x + t_begin : 0;
  const int len2 = live ? (int)min(T, n - t_begin) : 0;
  if constexpr (P1 == 2) {
    const int64_t start = (int64_t)c * XS.shift + XS.q0;  // may be < 0 for c = 0
    const bool need = c + 1 < C;                          // last chunk: state unused
    s_in[c] = need ? b * XS.ld + start : 0;
    s_lo[c] = need ? (int)max((int64_t)0, -start) : 0;
    // Only the rows that meet a tap: a non-finite sample past them must not
    // reach this chunk's state (0 * inf = NaN; it first meets a later chunk).
    s_len[c] = need ? (int)max((int64_t)0, min(XS.span, XS.n - start)) : 0;
  } else {
    s_in[c] = in2;
    s_lo[c] = 0;
    s_len[c] = c + 1 < C ? len2 : 0;  // last chunk: state unused
  }
  // VM > 0 stores through a raw buffer based at this channel's output row.
  s_out[c] = live ? (VM > 0 ? 0 : b * ld_y) + t_begin : 0;
  const int r0 = wv * kWave;  // this wave's rows
  const Rows rows{s_in + r0, s_out + r0, s_len + r0, s_lo + r0};
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(y + b * ld_y, 0, (int)(n * 4), 0x00020000);
  // VM > 0: affine buffer addressing (AffIO); loads may read up to the next
  // multiple of 4 samples (inside the row pitch, as the vector fetch does).
  AffIO io1{}, io2{};
  if constexpr (VM > 0) {
    const __amdgpu_buffer_rsrc_t in2 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(x) + b * ld_x, 0, (int)(((n + 3) & ~3) * 4), 0x00020000);
    io2 = aff_rows(in2, T, 0, T, r0, lane);
    if constexpr (P1 == 2) {
      const __amdgpu_buffer_rsrc_t in1 = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(XS.xs) + b * XS.ld, 0, (int)(((XS.n + 3) & ~3) * 4), 0x00020000);
      io1 = aff_rows(in1, XS.shift, XS.q0, T, r0, lane);
    } else {
      io1 = io2;
    }
  }

  double s1[S], s2[S], e[D];
#pragma unroll
  for (int k = 0; k < S; ++k) s1[k] = s2[k] = 0.0;
#pragma unroll
  for (int i = 0; i < D; ++i) e[i] = 0.0;

  // ---- pass 1: zero-state end state of the lane's chunk
  constexpr bool AFF = VM > 0;
  if constexpr (P1 == 2) {
    run_pass<S, kStateTable, kWave, VM, true, NORM, AFF>(XS.xs, y, rsrc, tile, rows, io1,
                                                         XS.rows, lane, s1, s2, e, p, G, clip);
  } else if constexpr (P1 == 1) {
    run_pass<S, kStateTable, kWave, VM, (VM > 0), NORM, AFF>(x, y, rsrc, tile, rows, io1, T,
                                                             lane, s1, s2, e, p, G, clip);
  } else {
    run_pass<S, kStateCascade, kWave, VM, (VM > 0), NORM, AFF>(x, y, rsrc, tile, rows, io1, T,
                                                               lane, s1, s2, e, p, G, clip);
#pragma unroll
    for (int k = 0; k < S; ++k) {
      e[2 * k] = s1[k];
      e[2 * k + 1] = s2[k];
    }
  }
  // A chunk whose input held an inf or NaN hands NaN on (nf_poison).
  nf_poison(e);

  // ---- carry scan
  block_sync<W>();  // W > 1: the scan slots overlap other waves' tiles
  s_in[c] = in2;  // pass-2 rows; pass 2 opens with a hand-off
  s_lo[c] = 0;
  s_len[c] = len2;
  carry_scan<S, W>(scan, e, s1, s2, sp, c, C);

  // ---- pass 2: outputs from the carried state
  run_pass<S, kApply, kWave, VM, (VM > 0), NORM, AFF>(x, y, rsrc, tile, rows, io2, T, lane, s1,
                                                      s2, e, p, G, clip);
}

// ---------------------------------------------------------------------------
// General path (C > kCB or S > 8): separate pass / carry launches.
// ---------------------------------------------------------------------------
template <int S, bool APPLY, bool NORM>
__global__ __launch_bounds__(kNT) void k_iir_pass(
    const float* __restrict__ x, float* __restrict__ y, int64_t n, int64_t ld_x,
    int64_t ld_y, SosParams p, int64_t C, int64_t T, int64_t lanes,
    const double* __restrict__ s_init, double* __restrict__ e_out, int clip, int vec_x,
    int vec_y) {
  constexpr int SS = S > 0 ? S : 1;
  __shared__ __attribute__((aligned(16))) float tile[kNT * kRow];
  __shared__ int64_t s_in[kNT], s_out[kNT];
  __shared__ int s_len[kNT], s_lo[kNT];
  const int tid = threadIdx.x;
  const int64_t g = (int64_t)blockIdx.x * kNT + tid;
  const int64_t cl = APPLY ? C : C - 1;  // chunks per channel handled here
  const bool live = g < lanes;
  int64_t b = 0, ch = 0;
  if (live) {
    b = g / cl;
    ch = g - b * cl;
  }
  const int64_t t_begin = ch * T;
  s_in[tid] = b * ld_x + t_begin;
  s_out[tid] = b * ld_y + t_begin;
  s_len[tid] = live ? (int)min(T, n - t_begin) : 0;
  s_lo[tid] = 0;
  const Rows rows{s_in, s_out, s_len, s_lo};

  double s1[SS], s2[SS], e[S > 0 ? 2 * S : 1];
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
  // Rows span many channels here: guarded loads and stores (VM 0).
  const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(y, 0, 0, 0x00020000);
  if (vec_x)
    run_pass<S, APPLY ? kApply : kStateCascade, kNT, 0, true, NORM>(x, y, none, tile, rows,
                                                                    AffIO{}, T, tid, s1, s2, e,
                                                                    p, nullptr, clip);
  else
    run_pass<S, APPLY ? kApply : kStateCascade, kNT, 0, false, NORM>(x, y, none, tile, rows,
                                                                     AffIO{}, T, tid,
                                                               s1, s2, e, p, nullptr, clip);
  if (!APPLY && live) {
    double* eo = e_out + g * (2 * S);
    double ev[2 * SS];
#pragma unroll
    for (int k = 0; k < SS; ++k) {
      ev[2 * k] = s1[k];
      ev[2 * k + 1] = s2[k];
    }
    nf_poison(ev);  // a chunk whose input held an inf or NaN hands NaN on
#pragma unroll
    for (int k = 0; k < S; ++k) {
      eo[2 * k] = ev[2 * k];
      eo[2 * k + 1] = ev[2 * k + 1];
    }
  }
}

// One lane per channel: S_0 = 0, S_{c+1} = P S_c + E_c.  The state vectors
// live in LDS ([D][256] doubles, double-buffered) so the kernel stays small for
// every D.
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
// square-and-multiply in float64 inside one workgroup (general path; the fused
// path gets A^T from the host as a kernel argument).
__global__ __launch_bounds__(1024) void k_iir_prep(SosParams p, int S, int64_t T,
                                                  double* __restrict__ P_out) {
  __shared__ double sA[32 * 32], sR[32 * 32], sTmp[32 * 32];
  const int D = 2 * S;
  const int tid = threadIdx.x;
  if (tid < D) {
    double X[32];
    for (int i = 0; i < D; ++i) X[i] = (i == tid) ? 1.0 : 0.0;
    cascade_state_step(p, S, false, X, 0.0);
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

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
size_t align256(size_t v) { return v > SIZE_MAX - 255 ? SIZE_MAX : (v + 255) & ~(size_t)255; }

struct WsLayout {
  size_t p_off, e_off, s_off, total;
};

bool fused_ok(int S, int64_t C, int64_t T) {
  return S >= 1 && S <= 8 && S != 7 && C >= 2 && C <= kCBMax && T % kTS == 0;
}

WsLayout ws_layout(int64_t B, int64_t n, int S, int64_t T) {
  WsLayout w{0, 0, 0, 0};
  const int64_t C = (S == 0 || T <= 0) ? 1 : ceil_div(n, T);
  if (C <= 1 || fused_ok(S, C, T)) return w;
  const size_t D = 2 * (size_t)S;
  w.p_off = 0;
  w.e_off = align256(D * D * sizeof(double));
  const size_t e_bytes = mul_sat((size_t)B, (size_t)(C - 1), D, sizeof(double));
  const size_t s_bytes = mul_sat((size_t)B, (size_t)C, D, sizeof(double));
  if (e_bytes == SIZE_MAX || s_bytes == SIZE_MAX) {
    w.total = SIZE_MAX;
    return w;
  }
  w.s_off = add_sat(w.e_off, align256(e_bytes));
  w.total = add_sat(w.s_off, align256(s_bytes));
  return w;
}

int padded_stages(int S) {
  if (S == 7) return 8;
  if (S > 8 && S <= 12) return 12;
  if (S > 12) return 16;
  return S;
}

template <int S>
int run_fused(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x, int64_t ld_y,
              const SosParams& p, bool norm, int clip, int64_t T, const double* G, int p1mode,
              int vec_x, int vec_y, const XState& XS, hipStream_t s) {
  static_assert(2 * S <= 16, "scan matrix is at most 16 x 16");
  ScanParams sp;
  const std::vector<double> P = chunk_transition(p, S, T);
  for (size_t i = 0; i < P.size(); ++i) sp.P[i] = P[i];
  const int C = (int)ceil_div(n, T);
  TraceScope trace(p1mode == 2 ? "iir_xstate" : "iir_fused", s);
  // VM: 1 = aligned rows of a length that is a multiple of 4, 2 = aligned rows
  // ending in a partial vector, 0 = any other pitch.  The buffer-store modes
  // address one channel's row with a 31-bit byte offset.
  const bool span_ok = n * 4 + 16 < (int64_t)kOob && (p1mode != 2 || XS.n * 4 + 16 < (int64_t)kOob);
  const int VMr = (vec_x && vec_y && span_ok) ? ((n % 4 == 0) ? 1 : 2) : 0;
  const dim3 grid((unsigned)B);
  const int W = C <= kWave ? 1 : C <= 2 * kWave ? 2 : 4;
#define DSP_WAVE_LAUNCH(P1v, VMv, NV)                                                         \
  do {                                                                                        \
    if (W == 1)                                                                               \
      hipLaunchKernelGGL((k_iir_wave<S, P1v, VMv, NV, 1>), grid, dim3(kWave), 0, s, x, y, B,  \
                         n, ld_x, ld_y, p, sp, G, T, C, clip, XS);                            \
    else if (W == 2)                                                                          \
      hipLaunchKernelGGL((k_iir_wave<S, P1v, VMv, NV, 2>), grid, dim3(2 * kWave), 0, s, x, y, \
                         B, n, ld_x, ld_y, p, sp, G, T, C, clip, XS);                         \
    else                                                                                      \
      hipLaunchKernelGGL((k_iir_wave<S, P1v, VMv, NV, 4>), grid, dim3(4 * kWave), 0, s, x, y, \
                         B, n, ld_x, ld_y, p, sp, G, T, C, clip, XS);                         \
  } while (0)
#define DSP_WAVE_VM(P1v, NV)                         \
  if (VMr == 1) DSP_WAVE_LAUNCH(P1v, 1, NV);         \
  else if (VMr == 2) DSP_WAVE_LAUNCH(P1v, 2, NV);    \
  else DSP_WAVE_LAUNCH(P1v, 0, NV);
  // The state tables are built for the NORM realisation (the EQ's); a cascade
  // with some b0 == 0 runs pass 1 as the cascade itself.
  if (!norm) { DSP_WAVE_VM(0, false) }
  else if (p1mode == 2) { DSP_WAVE_VM(2, true) }
  else if (p1mode == 1) { DSP_WAVE_VM(1, true) }
  else { DSP_WAVE_VM(0, true) }
#undef DSP_WAVE_VM
#undef DSP_WAVE_LAUNCH
  DSP_LAUNCHED("k_iir_wave");
  return DSP_OK;
}

template <int S, bool NORM>
int run_general(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x, int64_t ld_y,
                const SosParams& p, int clip, int64_t T, void* ws, int vec_x, int vec_y,
                hipStream_t s) {
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
      hipLaunchKernelGGL((k_iir_pass<S, false, NORM>), dim3((unsigned)ceil_div(lanes1, kNT)),
                         dim3(kNT), 0, s, x, y, n, ld_x, ld_y, p, C, T, lanes1,
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
    hipLaunchKernelGGL((k_iir_pass<S, true, NORM>), dim3((unsigned)ceil_div(lanes2, kNT)),
                       dim3(kNT), 0, s, x, y, n, ld_x, ld_y, p, C, T, lanes2, SI,
                       (double*)nullptr, clip, vec_x, vec_y);
  }
  DSP_LAUNCHED("k_iir_pass<apply>");
  return DSP_OK;
}

template <int S>
int run_cascade(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x, int64_t ld_y,
                const SosParams& p, bool norm, int clip, int64_t T, const double* G, void* ws,
                hipStream_t s) {
  const int vec_x = ((ld_x & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0);
  const int vec_y = ((ld_y & 3) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0);
  const int64_t C = (S == 0) ? 1 : ceil_div(n, T);
  if constexpr (S >= 1 && S <= 8 && S != 7) {
    if (fused_ok(S, C, T))
      return run_fused<S>(x, y, B, n, ld_x, ld_y, p, norm, clip, T, G, G ? 1 : 0, vec_x, vec_y,
                          XState{}, s);
  }
  if (norm) return run_general<S, true>(x, y, B, n, ld_x, ld_y, p, clip, T, ws, vec_x, vec_y, s);
  return run_general<S, false>(x, y, B, n, ld_x, ld_y, p, clip, T, ws, vec_x, vec_y, s);
}

}  // namespace

int xstate_geometry(int64_t chunk_len, int K, int L, int M, int64_t c, int64_t* shift,
                    int64_t* q0, int64_t* rows, int64_t* span_out) {
  DSP_REQUIRE(chunk_len > 0 && K >= 1 && L >= 1 && M >= 1 && c >= 0, "bad SRC/chunk geometry");
  DSP_REQUIRE(chunk_len <= ((int64_t)1 << 40) && L <= (1 << 24) && M <= (1 << 24) &&
                  c <= ((int64_t)1 << 40),
              "SRC/chunk geometry out of range");
  DSP_REQUIRE((chunk_len * M) % L == 0, "chunk_len*M=%lld is not a multiple of L=%d",
              (long long)(chunk_len * M), L);
  const int64_t sh = chunk_len * M / L;
  DSP_REQUIRE(sh % 4 == 0, "chunk input shift %lld is not a multiple of 4", (long long)sh);
  // q' of output t = 0..T-1 and tap k = 0..K-1: (t*M + c - k) / L where divisible.
  auto floor_div = [](int64_t a, int64_t d) { return a >= 0 ? a / d : -((-a + d - 1) / d); };
  const int64_t qmax = floor_div((chunk_len - 1) * M + c, L);
  const int64_t qmin = -floor_div(K - 1 - c, L);  // ceil((c - K + 1) / L)
  // Row starts c*shift + q0 on 128-byte boundaries when shift is a multiple of
  // 32 (config 3): a misaligned 128-byte row segment costs two cache lines.
  const int64_t lo = floor_div(qmin, 32) * 32;
  const int64_t span = qmax - lo + 1;
  *shift = sh;
  *q0 = lo;
  *rows = ceil_div(span, kTS) * kTS;
  if (span_out) *span_out = span;
  return DSP_OK;
}

bool xstate_applicable(int64_t n, int S, int64_t chunk_len, const float* xs, int64_t ld_xs,
                       int L, int M) {
  if (S < 1 || S > 8 || S == 7 || chunk_len <= 0 || chunk_len % kTS) return false;
  if ((chunk_len * M) % L || ((chunk_len * M) / L) % 4) return false;
  if ((ld_xs & 3) || (reinterpret_cast<uintptr_t>(xs) & 15)) return false;
  return fused_ok(S, ceil_div(n, chunk_len), chunk_len);
}

int launch_biquad_xstate(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x,
                         int64_t ld_y, const double* sos, int S, int clip, int64_t chunk_len,
                         const float* xs, int64_t n_in, int64_t ld_xs, int K, int L, int M,
                         int64_t c, const double* gx, int64_t gx_rows, hipStream_t s) {
  DSP_REQUIRE(S >= 1 && S <= 8 && S != 7, "x-domain states need 1 <= S <= 8, S != 7 (S=%d)", S);
  DSP_REQUIRE(fused_ok(S, ceil_div(n, chunk_len), chunk_len),
              "x-domain states need the fused cascade (n=%lld chunk_len=%lld)", (long long)n,
              (long long)chunk_len);
  XState XS{xs, ld_xs, n_in, 0, 0, 0, 0};
  if (int rc = xstate_geometry(chunk_len, K, L, M, c, &XS.shift, &XS.q0, &XS.rows, &XS.span))
    return rc;
  DSP_REQUIRE(gx_rows == XS.rows, "x-domain state table has %lld rows, geometry needs %lld",
              (long long)gx_rows, (long long)XS.rows);
  DSP_REQUIRE(x && y && sos && xs && gx, "null pointer");
  DSP_REQUIRE((ld_xs & 3) == 0 && (reinterpret_cast<uintptr_t>(xs) & 15) == 0 && ld_xs >= n_in,
              "x-domain states need 16-byte aligned SRC input rows");
  SosParams p;
  DSP_REQUIRE(realize(sos, S, &p), "x-domain states need every b0 != 0");
  const int vec_x = ((ld_x & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0);
  const int vec_y = ((ld_y & 3) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0);
  const int64_t T = chunk_len;
  switch (S) {
    case 1: return run_fused<1>(x, y, B, n, ld_x, ld_y, p, true, clip, T, gx, 2, vec_x, vec_y,
                                    XS, s);
    case 2: return run_fused<2>(x, y, B, n, ld_x, ld_y, p, true, clip, T, gx, 2, vec_x, vec_y,
                                    XS, s);
    case 3: return run_fused<3>(x, y, B, n, ld_x, ld_y, p, true, clip, T, gx, 2, vec_x, vec_y,
                                    XS, s);
    case 4: return run_fused<4>(x, y, B, n, ld_x, ld_y, p, true, clip, T, gx, 2, vec_x, vec_y,
                                    XS, s);
    case 5: return run_fused<5>(x, y, B, n, ld_x, ld_y, p, true, clip, T, gx, 2, vec_x, vec_y,
                                    XS, s);
    case 6: return run_fused<6>(x, y, B, n, ld_x, ld_y, p, true, clip, T, gx, 2, vec_x, vec_y,
                                    XS, s);
    case 8: return run_fused<8>(x, y, B, n, ld_x, ld_y, p, true, clip, T, gx, 2, vec_x, vec_y,
                                    XS, s);
    default: return set_error(DSP_EINVAL, "unsupported stage count %d", S);
  }
}

size_t biquad_workspace_bytes(int64_t B, int64_t n, int S, int64_t chunk_len) {
  if (B <= 0 || n <= 0 || S < 0 || S > DSP_MAX_STAGES || chunk_len <= 0) return 0;
  return ws_layout(B, n, padded_stages(S), chunk_len).total;
}

int launch_biquad(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x,
                  int64_t ld_y, const double* sos, int S, int clip, int64_t chunk_len,
                  const double* state_table, void* ws, size_t ws_bytes, hipStream_t s) {
  DSP_REQUIRE(B >= 0 && n >= 0, "bad sizes");
  DSP_REQUIRE(S >= 0 && S <= DSP_MAX_STAGES, "S=%d outside [0, %d]", S, DSP_MAX_STAGES);
  DSP_REQUIRE(chunk_len > 0 && chunk_len % kTS == 0,
              "chunk_len=%lld must be a positive multiple of %d", (long long)chunk_len, kTS);
  DSP_REQUIRE(chunk_len <= (int64_t)1 << 30, "chunk_len too large");
  DSP_REQUIRE(ld_x >= n && ld_y >= n, "leading dimension too small");
  if (B == 0 || n == 0) return DSP_OK;
  DSP_REQUIRE(x && y, "null pointer");
  DSP_REQUIRE(S == 0 || sos, "null sos");
  // Pad S up to an instantiated size with exact identity stages.
  const int Sp = padded_stages(S);
  SosParams p;
  const bool norm = realize(sos, S, &p);
  const size_t need = ws_layout(B, n, Sp, chunk_len).total;
  DSP_REQUIRE(ws_bytes >= need, "workspace too small: %zu < %zu bytes", ws_bytes, need);
  DSP_REQUIRE(need == 0 || ws, "null workspace");
  // The state-response table is laid out for exactly S stages.
  const double* G = (Sp == S) ? state_table : nullptr;
  switch (Sp) {
    case 0: return run_cascade<0>(x, y, B, n, ld_x, ld_y, p, norm, clip, chunk_len, G, ws, s);
    case 1: return run_cascade<1>(x, y, B, n, ld_x, ld_y, p, norm, clip, chunk_len, G, ws, s);
    case 2: return run_cascade<2>(x, y, B, n, ld_x, ld_y, p, norm, clip, chunk_len, G, ws, s);
    case 3: return run_cascade<3>(x, y, B, n, ld_x, ld_y, p, norm, clip, chunk_len, G, ws, s);
    case 4: return run_cascade<4>(x, y, B, n, ld_x, ld_y, p, norm, clip, chunk_len, G, ws, s);
    case 5: return run_cascade<5>(x, y, B, n, ld_x, ld_y, p, norm, clip, chunk_len, G, ws, s);
    case 6: return run_cascade<6>(x, y, B, n, ld_x, ld_y, p, norm, clip, chunk_len, G, ws, s);
    case 8: return run_cascade<8>(x, y, B, n, ld_x, ld_y, p, norm, clip, chunk_len, G, ws, s);
    case 12: return run_cascade<12>(x, y, B, n, ld_x, ld_y, p, norm, clip, chunk_len, G, ws, s);
    case 16: return run_cascade<16>(x, y, B, n, ld_x, ld_y, p, norm, clip, chunk_len, G, ws, s);
    default: return set_error(DSP_EINVAL, "unsupported stage count %d", S);
  }
}

}  // namespace dsp
