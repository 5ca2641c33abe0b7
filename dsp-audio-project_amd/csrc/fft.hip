// Batched FFT and windowed magnitude spectrum for gfx950: Stockham autosort
// passes of radix 16 held in registers, one LDS exchange per pass.
//
// Replaces reference modules/dsp_core.py:41-66 (fft_diezmado_en_tiempo, a
// recursive radix-2 DIT in pure Python: 2N-1 calls, each building exp(-2j*pi*k/N)
// and concatenating E + W*O, E - W*O) and dsp_core.py:74-98
// (calcular_espectro_magnitud: centre segment or zero-padded input, Hann window,
// FFT, |X[k]| for k <= N/2).  The DFT it computes is the same (natural-order
// X[k] = sum_n x[n] W_N^(nk)); only the factorisation differs.
//
// Algorithm (per transform of N = 2^log2n points):
//   passes p = 0..P-1 with radices R_p (16, except a first pass of 2, 4 or 8
//   when log2n is not a multiple of 4) and Ns = R_0 * ... * R_(p-1):
//     for every butterfly j < N/R_p, with m = j mod Ns:
//       v[r] = in[j + r*N/R_p] * W_N^(m*r*N/(Ns*R_p))      r < R_p
//       v    = DFT_R(v)                                    (registers)
//       out[(j - m)*R_p + m + r*Ns] = v[r]
//   The output is in natural order after the last pass (Stockham autosort).
// A radix-16 pass is a 4 x 4 split with compile-time W_16 constants, so a
// 4096-point transform is 3 LDS round trips instead of the 12 stages of a
// radix-2 kernel.  The first pass reads HBM directly (window and zero padding
// applied on load) and the last pass writes HBM directly (index j + r*Ns:
// coalesced), so the transform touches LDS P-1 times.
//
// LDS: one padded buffer per transform, element i at i + (i >> 4): pass-0
// writes (stride R) and the strided reads then spread over the 64 banks.
// Twiddles: w1 = W_N^(m*N/(Ns*R)) from the caller's fp64-computed table
// exp(-2*pi*i*k/N), k < N/2 (rounded to fp32), and w_r = w1^r by at most four
// complex products (error ~4 ulp, far inside the 1e-5 tolerance).
// Small transforms (N < 4096) pack 256 / (N/16) transforms per workgroup.
// The spectrum mode also runs a framed STFT: transform t = (row, frame) reads
// the window-weighted frame starting hop*frame samples into the row's segment.
#include "common.h"

namespace dsp {
namespace {

enum FftMode { kC2C = 0, kR2C = 1, kSpec = 2 };

typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float2 cadd(float2 a, float2 b) {
  return make_float2(a.x + b.x, a.y + b.y);
}
__device__ __forceinline__ float2 csub(float2 a, float2 b) {
  return make_float2(a.x - b.x, a.y - b.y);
}
__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
  return make_float2(fmaf(a.x, w.x, -a.y * w.y), fmaf(a.x, w.y, a.y * w.x));
}

// Complex values as 2-float vectors: every add, product and fma below is one
// v_pk_*_f32 (a complex product is a pk_mul and a pk_fma with operand
// swizzles), half the VALU instructions of the float2-struct code.
typedef float pf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ pf2 pcmul(pf2 a, pf2 w) { return a.xx * w + a.yy * pf2{-w.y, w.x}; }
__device__ __forceinline__ pf2 pmi(pf2 a) { return pf2{a.y, -a.x}; }  // a * (-i)

// The same with register operands, spelled out: the compiler builds the
// swapped, negated copy of w ({-w.y, w.x}) with a move and an xor, where the
// VOP3P operand selects and negations do it for free.
//   a * w:      t = (a.x w.x, a.x w.y);  r = t + (-a.y w.y, a.y w.x)
//   s + d * w:  the same with s as the first accumulator
//   t -+ i d:   (t.x +- d.y, t.y -+ d.x)  (t + (-i) d and t - (-i) d)
__device__ __forceinline__ pf2 vcmul(pf2 a, pf2 w) {
  pf2 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(w));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
      : "=v"(r) : "v"(a), "v"(w), "v"(t));
  return r;
}
__device__ __forceinline__ pf2 vcfma(pf2 d, pf2 w, pf2 s) {
  pf2 t, r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(t) : "v"(d), "v"(w), "v"(s));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
      : "=v"(r) : "v"(d), "v"(w), "v"(t));
  return r;
}
__device__ __forceinline__ pf2 vadd_mi(pf2 t, pf2 d) {
  pf2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(t), "v"(d));
  return r;
}
__device__ __forceinline__ pf2 vsub_mi(pf2 t, pf2 d) {
  pf2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(t), "v"(d));
  return r;
}


// Variable-twiddle products and the radix-4 butterfly through the packed
// helpers above (the float2 expressions made the compiler build each swapped,
// negated twiddle copy with a move and an xor).
__device__ __forceinline__ float2 cmulv(float2 a, float2 w) {
  const pf2 r = vcmul(pf2{a.x, a.y}, pf2{w.x, w.y});
  return make_float2(r.x, r.y);
}

// |v|.  sqrtf is correctly rounded, which the compiler expands around
// v_sqrt_f32 into ~14 instructions (denormal scaling and a two-sided fma
// correction); the bare instruction is within 1 ulp, 2^-23 relative, far inside
// the spectra's 1e-5 tolerance, and drops ~450 of the ~2900 VALU instructions
// a 4096-point magnitude spectrum takes per wave.
__device__ __forceinline__ float cabsf_(float2 v) {
  const float p = fmaf(v.x, v.x, v.y * v.y);
  return __builtin_amdgcn_sqrtf(p);
}

// a * W_16^q for a compile-time q (after unrolling); exact for q % 4 == 0.
__device__ __forceinline__ float2 w16mul(float2 a, int q) {
  constexpr float c1 = 0.92387953251128674f;  // cos(pi/8)
  constexpr float s1 = 0.38268343236508977f;  // sin(pi/8)
  constexpr float h = 0.70710678118654752f;   // sqrt(1/2)
  switch (q & 15) {
    case 0: return a;
    case 1: return cmul(a, make_float2(c1, -s1));
    case 2: return cmul(a, make_float2(h, -h));
    case 3: return cmul(a, make_float2(s1, -c1));
    case 4: return make_float2(a.y, -a.x);
    case 5: return cmul(a, make_float2(-s1, -c1));
    case 6: return cmul(a, make_float2(-h, -h));
    case 7: return cmul(a, make_float2(-c1, -s1));
    case 8: return make_float2(-a.x, -a.y);
    case 9: return cmul(a, make_float2(-c1, s1));
    case 10: return cmul(a, make_float2(-h, h));
    case 11: return cmul(a, make_float2(-s1, c1));
    case 12: return make_float2(-a.y, a.x);
    case 13: return cmul(a, make_float2(s1, c1));
    case 14: return cmul(a, make_float2(h, h));
    default: return cmul(a, make_float2(c1, s1));
  }
}

__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
  const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
  const float2 t2 = cadd(a1, a3), d = csub(a1, a3);
  a0 = cadd(t0, t2);
  a2 = csub(t0, t2);
  const pf2 r1 = vadd_mi(pf2{t1.x, t1.y}, pf2{d.x, d.y});  // t1 + (a1 - a3) * (-i)
  const pf2 r3 = vsub_mi(pf2{t1.x, t1.y}, pf2{d.x, d.y});
  a1 = make_float2(r1.x, r1.y);
  a3 = make_float2(r3.x, r3.y);
}

// In-place forward DFT of R points, natural order in and out.
template <int R>
__device__ __forceinline__ void dft(float2 (&v)[R]) {
  if constexpr (R == 2) {
    const float2 a = v[0];
    v[0] = cadd(a, v[1]);
    v[1] = csub(a, v[1]);
  } else if constexpr (R == 4) {
    dft4(v[0], v[1], v[2], v[3]);
  } else if constexpr (R == 8) {
    // n = 2 n1 + n2, k = k1 + 4 k2
    dft4(v[0], v[2], v[4], v[6]);
    dft4(v[1], v[3], v[5], v[7]);
    float2 o[8];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      const float2 y0 = v[2 * k1], y1 = w16mul(v[2 * k1 + 1], 2 * k1);
      o[k1] = cadd(y0, y1);
      o[k1 + 4] = csub(y0, y1);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = o[i];
  } else if constexpr (R == 16) {
    // n = 4 n1 + n2, k = k1 + 4 k2
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4(v[n2], v[4 + n2], v[8 + n2], v[12 + n2]);
    // Y[n2][k1] sits at v[4 k1 + n2]
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1)
#pragma unroll
      for (int n2 = 1; n2 < 4; ++n2) v[4 * k1 + n2] = w16mul(v[4 * k1 + n2], n2 * k1);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) dft4(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
    float2 o[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) o[k1 + 4 * k2] = v[4 * k1 + k2];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = o[i];
  }
}

// ---------------------------------------------------------------------------
// Compile-time plan
// ---------------------------------------------------------------------------
template <int LOG2N>
struct Plan {
  static constexpr int N = 1 << LOG2N;
  static constexpr int NP = LOG2N == 0 ? 0 : (LOG2N + 3) / 4;
  static constexpr int RMAX = LOG2N >= 4 ? 16 : N;
  static constexpr int TPT = N / RMAX;                      // threads per transform
  static constexpr int TPB = TPT >= 256 ? 1 : 256 / TPT;    // transforms per block
  static constexpr int NT = TPB * TPT;
  static constexpr int PADN = N + (N >> 4);
  static constexpr int radix(int p) {
    return (p == 0 && (LOG2N & 3) != 0) ? (1 << (LOG2N & 3)) : RMAX;
  }
  static constexpr int ns(int p) { return p == 0 ? 1 : ns(p - 1) * radix(p - 1); }
};

__device__ __forceinline__ int lpad(int i) { return i + (i >> 4); }

struct FftArgs {
  const float* in;     // real rows (kR2C, kSpec) or interleaved complex rows (kC2C)
  float* out;          // complex rows (kC2C, kR2C) or magnitudes (kSpec)
  int64_t B, ld_in, ld_out;      // B = transforms (rows x frames for kSpec)
  int64_t seg_start, seg_len;    // kSpec: valid samples [seg_start, seg_start + seg_len)
  int64_t hop, frames;           // kSpec: frame f of a row starts hop*f after seg_start
  const float* win;              // kSpec
  const float2* tw;              // exp(-2 pi i k / N), k < N/2
};

// Where transform t reads its input: element n is in[base + n] (complex or real
// element units); kSpec frames also carry their valid length.
struct InRow {
  int64_t base;
  int64_t valid;  // kSpec: samples of the frame inside the segment
};

template <int MODE>
__device__ __forceinline__ InRow in_row(const FftArgs& a, int64_t t) {
  if constexpr (MODE == kSpec) {
    const int64_t row = a.frames == 1 ? t : t / a.frames;
    const int64_t f0 = (t - row * a.frames) * a.hop;  // frame start within the segment
    return InRow{row * a.ld_in + a.seg_start + f0, a.seg_len - f0};
  } else {
    return InRow{t * a.ld_in, 0};
  }
}

// Value n of the transform as the first pass reads it.
template <int MODE>
__device__ __forceinline__ float2 load_input(const FftArgs& a, const InRow& r, int n, bool live) {
  if (!live) return make_float2(0.f, 0.f);
  if constexpr (MODE == kC2C) {
    return reinterpret_cast<const float2*>(a.in)[r.base + n];
  } else if constexpr (MODE == kR2C) {
    return make_float2(a.in[r.base + n], 0.f);
  } else {
    const float s = (n < r.valid) ? a.in[r.base + n] : 0.f;
    return make_float2(s * a.win[n], 0.f);
  }
}

template <int MODE, int N>
__device__ __forceinline__ void store_output(const FftArgs& a, int64_t t, int k, float2 v,
                                             bool live) {
  if (!live) return;
  if constexpr (MODE == kSpec) {
    if (k <= N / 2) a.out[t * a.ld_out + k] = cabsf_(v);
  } else {
    reinterpret_cast<float2*>(a.out)[t * a.ld_out + k] = v;
  }
}

// w1 of every butterfly of pass P (the twiddle loads are issued before pass 0 so
// their latency hides under it instead of after each barrier).
template <int LOG2N, int P>
struct Tw {
  float2 w[Plan<LOG2N>::NP > P + 1 ? Plan<LOG2N>::RMAX / Plan<LOG2N>::radix(P + 1) : 1];
  Tw<LOG2N, P + 1> next;
};
template <int LOG2N>
struct Tw<LOG2N, 15> {};

// tstr: stride into the caller's table (2 when the table is for 2N points,
// N_total / N for a sub-transform of a four-step FFT).
template <int LOG2N, int P>
__device__ __forceinline__ void load_tw(Tw<LOG2N, P>& tw, const float2* __restrict__ table,
                                        int j0, int64_t tstr = 1) {
  using PL = Plan<LOG2N>;
  if constexpr (P + 1 < PL::NP) {
    constexpr int R = PL::radix(P + 1);
    constexpr int NS = PL::ns(P + 1);
#pragma unroll
    for (int b = 0; b < PL::RMAX / R; ++b) {
      const int m = (j0 + b * PL::TPT) & (NS - 1);
      tw.w[b] = table[(int64_t)m * (PL::N / (NS * R)) * tstr];
    }
    load_tw<LOG2N, P + 1>(tw.next, table, j0, tstr);
  }
}

// IO policies of a transform: load(n) feeds the first pass, store(k, v) takes
// the last pass's natural-order output.  kLdsIn: load() reads the LDS buffer
// the passes work in, so the first pass also waits before writing.
template <int MODE, int N>
struct GlobalIO {
  static constexpr bool kLdsIn = false;
  const FftArgs& a;
  InRow ir;
  int64_t t;
  bool live;
  __device__ __forceinline__ float2 load(int n) const { return load_input<MODE>(a, ir, n, live); }
  __device__ __forceinline__ void store(int k, float2 v) const {
    store_output<MODE, N>(a, t, k, v, live);
  }
};

template <int LOG2N, int P, class IO, bool LOWREG = false>
__device__ __forceinline__ void run_pass(const IO& io, float2* buf, int j0,
                                         const Tw<LOG2N, P - 1 < 0 ? 0 : P - 1>& tw) {
  using PL = Plan<LOG2N>;
  constexpr int N = PL::N;
  constexpr int R = PL::radix(P);
  constexpr int NS = PL::ns(P);
  constexpr int NB = PL::RMAX / R;  // butterflies per thread
  constexpr int STRIDE = N / R;
  constexpr bool FIRST = P == 0, LAST = P == PL::NP - 1;
  float2 v[NB][R];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int j = j0 + b * PL::TPT;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int n = j + r * STRIDE;
      v[b][r] = FIRST ? io.load(n) : buf[lpad(n)];
    }
  }
  // every read of this pass precedes its (in-place) writes (a barrier for LDS
  // only: one that also drained global loads would wait out the four-step's
  // twiddle loads that are meant to be in flight under the passes)
  if constexpr (!FIRST || IO::kLdsIn) lds_barrier();
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int j = j0 + b * PL::TPT;
    const int m = j & (NS - 1);
    if constexpr (NS > 1 && !LOWREG) {
      float2 w[R];
      w[1] = tw.w[b];
#pragma unroll
      for (int r = 2; r < R; ++r) w[r] = (r & 1) ? cmulv(w[r - 1], w[1]) : cmulv(w[r / 2], w[r / 2]);
#pragma unroll
      for (int r = 1; r < R; ++r) v[b][r] = cmulv(v[b][r], w[r]);
    } else if constexpr (NS > 1) {
      // Few live registers: w1, w2, w4, w8 by squaring, w_r as the product of
      // the powers in r's binary digits, applied as soon as it is formed.
      float2 p2[4];
      p2[0] = tw.w[b];
#pragma unroll
      for (int e = 1; e < 4; ++e) p2[e] = cmulv(p2[e - 1], p2[e - 1]);
#pragma unroll
      for (int r = 1; r < R; ++r) {
        float2 w = make_float2(1.f, 0.f);
        bool first = true;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if ((r >> e) & 1) {
            w = first ? p2[e] : cmulv(w, p2[e]);
            first = false;
          }
        v[b][r] = cmulv(v[b][r], w);
      }
    }
    dft<R>(v[b]);
    const int base = (j - m) * R + m;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = base + r * NS;
      if constexpr (LAST) io.store(k, v[b][r]);
      else buf[lpad(k)] = v[b][r];
    }
  }
  if constexpr (!LAST) lds_barrier();
  if constexpr (P + 1 < PL::NP) {
    if constexpr (P == 0) run_pass<LOG2N, P + 1, IO, LOWREG>(io, buf, j0, tw);
    else run_pass<LOG2N, P + 1, IO, LOWREG>(io, buf, j0, tw.next);
  }
}

template <int LOG2N, int MODE>
__global__ __launch_bounds__(Plan<LOG2N>::NT) void k_fft(FftArgs a) {
  using PL = Plan<LOG2N>;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  const int tl = threadIdx.x / PL::TPT;
  const int j0 = threadIdx.x - tl * PL::TPT;
  const int64_t t = (int64_t)blockIdx.x * PL::TPB + tl;
  const bool live = t < a.B;
  const GlobalIO<MODE, PL::N> io{a, in_row<MODE>(a, live ? t : 0), t, live};
  if constexpr (PL::NP == 0) {
    io.store(0, io.load(0));
  } else {
    Tw<LOG2N, 0> tw;
    load_tw<LOG2N, 0>(tw, a.tw, j0);
    run_pass<LOG2N, 0>(io, lds + tl * PL::PADN, j0, tw);
  }
}

// ---------------------------------------------------------------------------
// Real-input magnitude spectrum (spectrum / STFT mode, N >= 32): the N real
// samples are packed as N/2 complex z[n] = x[2n] + i x[2n+1] (window applied),
// one N/2-point Stockham transform Z runs in LDS, and the split
//   E = (Z[k] + conj Z[N/2-k]) / 2,  O = (Z[k] - conj Z[N/2-k]) / (2i)
//   X[k] = E + W_N^k O,  X[N/2-k] = conj(E - W_N^k O)
// gives |X[k]| for every k <= N/2 from one (k, N/2-k) pair per thread: half the
// butterflies and half the LDS of the complex transform.
// ---------------------------------------------------------------------------
template <int NH>  // NH = N/2, the complex transform's size
struct RealSpecIO {
  static constexpr bool kLdsIn = false;
  const FftArgs& a;
  InRow ir;
  float2* buf;
  bool live;
  bool pairs;  // the frame's samples start 8-byte aligned: one float2 load per pair
  __device__ __forceinline__ float2 load(int n) const {
    if (!live) return make_float2(0.f, 0.f);
    const int i = 2 * n;
    if (pairs && i + 1 < ir.valid) {
      const float2 sv = *reinterpret_cast<const float2*>(a.in + ir.base + i);
      const float2 wv = reinterpret_cast<const float2*>(a.win)[n];
      return make_float2(sv.x * wv.x, sv.y * wv.y);
    }
    const float s0 = (i < ir.valid) ? a.in[ir.base + i] : 0.f;
    const float s1 = (i + 1 < ir.valid) ? a.in[ir.base + i + 1] : 0.f;
    return make_float2(s0 * a.win[i], s1 * a.win[i + 1]);
  }
  __device__ __forceinline__ void store(int k, float2 v) const { buf[lpad(k)] = v; }
};

template <int LOG2N>  // LOG2N of the real length N
__global__ __launch_bounds__(Plan<LOG2N - 1>::NT) void k_spec_real(FftArgs a) {
  using PL = Plan<LOG2N - 1>;
  constexpr int N = 1 << LOG2N, NH = N / 2;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  const int tl = threadIdx.x / PL::TPT;
  const int j0 = threadIdx.x - tl * PL::TPT;
  const int64_t t = (int64_t)blockIdx.x * PL::TPB + tl;
  const bool live = t < a.B;
  float2* buf = lds + tl * PL::PADN;
  Tw<LOG2N - 1, 0> tw;
  load_tw<LOG2N - 1, 0>(tw, a.tw, j0, 2);
  const InRow ir = in_row<kSpec>(a, live ? t : 0);
  const bool pairs = ((reinterpret_cast<uintptr_t>(a.in + ir.base) & 7) == 0) &&
                     ((reinterpret_cast<uintptr_t>(a.win) & 7) == 0);
  run_pass<LOG2N - 1, 0>(RealSpecIO<NH>{a, ir, buf, live, pairs}, buf, j0, tw);
  __syncthreads();  // the last pass stored Z into LDS
  if (!live) return;
  float* mr = a.out + t * a.ld_out;
  for (int k = j0; k <= NH / 2; k += PL::TPT) {
    const float2 zk = buf[lpad(k)];
    const float2 zm = buf[lpad((NH - k) & (NH - 1))];
    const float2 e = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
    const float2 o = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
    const float2 w = a.tw[k < NH ? k : 0];  // k = NH/2 < N/2 always; table holds W_N^k, k < N/2
    const float2 wo = cmulv(o, w);
    const float2 xk = cadd(e, wo), xm = csub(e, wo);
    mr[k] = cabsf_(xk);
    if (k > 0 && k < NH / 2) mr[NH - k] = cabsf_(xm);
    if (k == 0) mr[NH] = fabsf(zk.x - zk.y);
  }
}

template <int LOG2N>
int launch_spec_real(const FftArgs& a, hipStream_t s) {
  using PL = Plan<LOG2N - 1>;
  const size_t shm = (size_t)PL::TPB * PL::PADN * sizeof(float2);
  if (int rc = allow_lds(k_spec_real<LOG2N>, shm)) return rc;
  const unsigned grid = (unsigned)ceil_div(a.B, PL::TPB);
  hipLaunchKernelGGL(k_spec_real<LOG2N>, dim3(grid), dim3(PL::NT), shm, s, a);
  DSP_LAUNCHED("k_spec_real");
  return DSP_OK;
}

// Transform entirely in LDS (passes after the first, four-step sub-transforms).
template <int N>
struct LdsIO {
  static constexpr bool kLdsIn = true;
  float2* buf;
  __device__ __forceinline__ float2 load(int n) const { return buf[lpad(n)]; }
  __device__ __forceinline__ void store(int k, float2 v) const { buf[lpad(k)] = v; }
};

// ---------------------------------------------------------------------------
// Streaming magnitude spectrum (round 3; the default for N = 2^6 .. 2^14 with a
// first pass of radix < 16): the same real-input transform as k_spec_real,
// but a persistent grid in which every workgroup walks its transforms in a
// loop and keeps the next transform's segment in flight while the current one
// runs its LDS passes, with 16-byte loads:
//   * pass 0 is remapped so that thread j0 owns the NB0 consecutive
//     butterflies NB0*j0 .. NB0*j0+NB0-1 (pass 0 has no twiddles, so any
//     butterfly-to-thread map works): for every r its inputs are NB0
//     consecutive complex values = 2*NB0 consecutive real samples, i.e. NB0/2
//     float4 loads per lane, contiguous across the wave;
//   * the window (the same for every transform) is re-read from L1/L2;
//   * the prefetched float4s of transform t+G are issued right after the
//     window multiply of transform t, so HBM latency hides under t's LDS
//     passes and split (the round-2 kernel issued each transform's loads only
//     when its workgroup started: SQ_WAIT_ANY / SQ_WAVE_CYCLES = 0.71).
// Rows whose segment start is not 16-byte aligned, or frames past the
// segment's end, take per-sample guarded loads (same values).
// ---------------------------------------------------------------------------
template <int LOG2N>
struct SpecStream {
  using PL = Plan<LOG2N - 1>;                 // the N/2-point complex transform
  static constexpr int N = 1 << LOG2N, NH = N / 2;
  static constexpr int R0 = PL::radix(0);
  static constexpr int NB0 = PL::RMAX / R0;    // pass-0 butterflies per thread
  static constexpr int S0 = NH / R0;           // pass-0 input stride (complex)
  static constexpr int NQ = NB0 / 2;           // float4s per r
  static_assert(NB0 >= 2 && NB0 % 2 == 0, "pass 0 needs >= 2 butterflies per thread");
};

// The transform's pass-0 samples as float4s through a raw buffer resource
// over its frame: one VGPR offset for all loads (the r strides go to the
// SGPR/immediate offsets), and bytes past the frame's valid samples -- or the
// whole frame of a dead transform -- read as zeros (the hardware checks every
// dword against num_records), which is the zero padding of dsp_core.py:81-82.
template <int LOG2N>
__device__ __forceinline__ void spec_stream_load(const FftArgs& a, const InRow& ir, bool live,
                                                 int j0, f32x4_t (&raw)[SpecStream<LOG2N>::NQ]
                                                                         [SpecStream<LOG2N>::R0]) {
  using SS = SpecStream<LOG2N>;
  const int64_t valid = live ? (ir.valid < SS::N ? (ir.valid > 0 ? ir.valid : 0) : SS::N) : 0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.in) + (live ? ir.base : 0), 0, (int)(valid * 4), 0x00020000);
  const int vo = 4 * 2 * SS::NB0 * j0;  // bytes
#pragma unroll
  for (int r = 0; r < SS::R0; ++r)
#pragma unroll
    for (int q = 0; q < SS::NQ; ++q)
      raw[q][r] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 4 * 2 * (2 * q + r * SS::S0), 2);
}

constexpr int kSpecWaves = 3;  // waves per SIMD the streaming kernel is compiled for
constexpr int kSpecTpbx = 2;   // transforms per workgroup (1: same at 32768 ch, 8 % slower at 4096)
template <int LOG2N, int TPBX>
__global__ __launch_bounds__(TPBX * Plan<LOG2N - 1>::TPT)
__attribute__((amdgpu_waves_per_eu(kSpecWaves))) void k_spec_stream(FftArgs a, int64_t units) {
  using SS = SpecStream<LOG2N>;
  using PL = typename SS::PL;
  constexpr int NH = SS::NH, R0 = SS::R0, NB0 = SS::NB0, NQ = SS::NQ;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  int tl = threadIdx.x / PL::TPT;
  // A transform of >= 64 threads is whole waves: tl is wave-uniform, and saying
  // so keeps the frame's buffer resource in SGPRs (otherwise every buffer load
  // sits in a readfirstlane waterfall loop).
  if constexpr (PL::TPT % 64 == 0) tl = __builtin_amdgcn_readfirstlane(tl);
  const int j0 = threadIdx.x - tl * PL::TPT;
  float2* buf = lds + tl * PL::PADN;
  f32x4_t raw[NQ][R0];
  int64_t u = blockIdx.x;
  {
    const int64_t t = u * TPBX + tl;
    const bool live = u < units && t < a.B;
    spec_stream_load<LOG2N>(a, in_row<kSpec>(a, live ? t : 0), live, j0, raw);
  }
  for (; u < units; u += gridDim.x) {
    // An opaque copy of the thread's index per iteration: every LDS / table
    // address below depends only on it, and hoisting them out of the loop
    // costs ~120 VGPRs (206 vs 84 without the loop).
    int jj = j0;
    asm volatile("" : "+v"(jj));
    const int64_t t = u * TPBX + tl;
    const bool live = t < a.B;
    // window the transform's samples (packed even/odd as complex; the window
    // is re-read from L1/L2 here rather than held in 32 VGPRs across the
    // passes) ...
    // (opaque per-iteration table pointers: otherwise the loop-invariant
    // window and twiddle loads -- and the twiddle powers computed from them --
    // are hoisted out of the loop into ~100 VGPRs; they are L1 hits)
    const float* winp = a.win;
    const float2* twp = a.tw;
    asm volatile("" : "+s"(winp), "+s"(twp));
    Tw<LOG2N - 1, 0> tw;
    load_tw<LOG2N - 1, 0>(tw, twp, jj, 2);
    float2 v[NB0][R0];
#pragma unroll
    for (int r = 0; r < R0; ++r)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const f32x4_t w =
            *reinterpret_cast<const f32x4_t*>(winp + 2 * (NB0 * jj + 2 * q + r * SS::S0));
        const f32x4_t x = raw[q][r];
        v[2 * q][r] = make_float2(x.x * w.x, x.y * w.y);
        v[2 * q + 1][r] = make_float2(x.z * w.z, x.w * w.w);
      }
    // ... and put the next one in flight
    {
      const int64_t un = u + gridDim.x;
      const int64_t tn = un * TPBX + tl;
      const bool ln = un < units && tn < a.B;
      spec_stream_load<LOG2N>(a, in_row<kSpec>(a, ln ? tn : 0), ln, jj, raw);
    }
    // pass 0 (radix R0, no twiddles) into LDS in Stockham order
#pragma unroll
    for (int b = 0; b < NB0; ++b) {
      dft<R0>(v[b]);
      const int jb = NB0 * jj + b;
#pragma unroll
      for (int r = 0; r < R0; ++r) buf[lpad(jb * R0 + r)] = v[b][r];
    }
    __syncthreads();
    if constexpr (PL::NP > 1)
      run_pass<LOG2N - 1, 1, LdsIO<NH>, true>(LdsIO<NH>{buf}, buf, jj, tw);
    __syncthreads();  // the last pass stored Z into LDS
    if (live) {
      float* mr = a.out + t * a.ld_out;
      for (int k = jj; k <= NH / 2; k += PL::TPT) {
        const float2 zk = buf[lpad(k)];
        const float2 zm = buf[lpad((NH - k) & (NH - 1))];
        const float2 e = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
        const float2 o = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
        const float2 w = twp[k < NH ? k : 0];
        const float2 wo = cmulv(o, w);
        const float2 xk = cadd(e, wo), xm = csub(e, wo);
        mr[k] = cabsf_(xk);
        if (k > 0 && k < NH / 2) mr[NH - k] = cabsf_(xm);
        if (k == 0) mr[NH] = fabsf(zk.x - zk.y);
      }
    }
    __syncthreads();  // the split's LDS reads precede the next transform's pass 0
  }
}

template <int LOG2N>
int launch_spec_stream(const FftArgs& a, hipStream_t s) {
  using PL = Plan<LOG2N - 1>;
  constexpr int TPBX = kSpecTpbx;
  const size_t shm = (size_t)TPBX * PL::PADN * sizeof(float2);
  if (int rc = allow_lds(k_spec_stream<LOG2N, TPBX>, shm)) return rc;
  const int64_t units = ceil_div(a.B, TPBX);
  const int res = resident_groups<k_spec_stream<LOG2N, TPBX>>(TPBX * PL::TPT, shm);
  DSP_REQUIRE(res > 0, "occupancy query failed");
  const unsigned grid = (unsigned)(units < res ? units : res);
  hipLaunchKernelGGL((k_spec_stream<LOG2N, TPBX>), dim3(grid), dim3(TPBX * PL::TPT), shm, s, a,
                     units);
  DSP_LAUNCHED("k_spec_stream");
  return DSP_OK;
}

// ---------------------------------------------------------------------------
// One-wave 4096-point magnitude spectrum (round 3; the default for log2n = 12,
// the benchmark's n_fft).  A wave owns
// one transform at a time and never waits on another wave: the 2048 packed
// values c[n] = x[2n] w[2n] + i x[2n+1] w[2n+1] sit 32 per lane and the
// 2048-point transform is a 32 x 64 four-step split
//   n = 64 n1 + n2 (lane n2 holds n1 = 0..31),   k = k1 + 32 k2
//   A  B[n2][k1] = W_2048^(n2 k1) DFT32_n1(c[64 n1 + n2])         registers
//   T  lane L = 2 k1 + h takes Y[k1][2m + h], m < 32                LDS, 2 planes of 8 KB
//   B  F_h[j] = DFT32_m(...);  Z[k1 + 32 j] = F_0 + W_64^j F_1,
//      Z[k1 + 32 (j + 32)] = F_0 - W_64^j F_1                        registers + DPP pair swap
// so lane L ends with Z[K], K = k1 + 1024 h + 32 j (j < 32).  The real split
//   X[K] = s - i W_4096^K d,  s = Z[K] + conj Z[-K],  d = Z[K] - conj Z[-K]
// (with Z already halved: the 1/2 rides on the step-A twiddles) takes Z[-K]
// from lane (1 - L) mod 64, register 31 - j, by one bpermute per component;
// lanes 0 and 1, each other's partners at register 32 - j, take the previous
// bpermute's value (and their own Z at j = 0).  For fixed j, |X[K]| is two runs
// of 32 consecutive floats across the wave.  Per transform and lane: 32 sample
// loads (b64) and 5 twiddle loads, 32 window reads from the workgroup's LDS
// copy, 128 transpose accesses, 64 bpermutes, 64 DPP moves, 32 stores, no
// barrier: 35 % fewer VALU instructions than k_spec_stream's three LDS
// Stockham passes (which need a workgroup barrier each), DESIGN.md section 3.3.
// ---------------------------------------------------------------------------
// W_N^m for any m from the table exp(-2 pi i k / N), k < N/2.
__device__ __forceinline__ float2 tw_full(const float2* __restrict__ tw, int64_t m, int64_t N) {
  m &= N - 1;
  const float2 w = tw[m < N / 2 ? m : m - N / 2];
  return m < N / 2 ? w : make_float2(-w.x, -w.y);
}

constexpr int kWaveRow = 66;               // transpose row stride (floats): conflict-free both ways
constexpr int kWaveLds = 32 * kWaveRow;    // floats of LDS per wave
constexpr int kWavePerGroup = 16;         // one workgroup per CU (see k_spec_wave12)

// W_128^j = exp(-2 pi i j / 128) for a compile-time j in [0, 128).  oz: an
// opaque zero OR-ed into the bits, so that the constants are formed where they
// are used (SALU) instead of hoisted out of the caller's loop: hoisted, the
// wave kernel's ~100 constant SGPRs spilled through v_writelane/v_readlane,
// ~160 VALU instructions per transform.
__device__ __forceinline__ pf2 w128(int j, int oz = 0) {
  constexpr float c[33] = {
      1.000000000e+00f, 9.987954562e-01f, 9.951847267e-01f, 9.891765100e-01f,
      9.807852804e-01f, 9.700312532e-01f, 9.569403357e-01f, 9.415440652e-01f,
      9.238795325e-01f, 9.039892931e-01f, 8.819212643e-01f, 8.577286100e-01f,
      8.314696123e-01f, 8.032075315e-01f, 7.730104534e-01f, 7.409511254e-01f,
      7.071067812e-01f, 6.715589548e-01f, 6.343932842e-01f, 5.956993045e-01f,
      5.555702330e-01f, 5.141027442e-01f, 4.713967368e-01f, 4.275550934e-01f,
      3.826834324e-01f, 3.368898534e-01f, 2.902846773e-01f, 2.429801799e-01f,
      1.950903220e-01f, 1.467304745e-01f, 9.801714033e-02f, 4.906767433e-02f,
      0.0f};  // cos(pi j / 64)
  const float sgn = j < 64 ? 1.f : -1.f;  // W_128^(j+64) = -W_128^j
  j &= 63;
  const float cs = j <= 32 ? c[j] : -c[64 - j];
  const float sn = j <= 32 ? c[32 - j] : c[j - 32];
  return pf2{__int_as_float(__float_as_int(sgn * cs) | oz),
             __int_as_float(__float_as_int(-sgn * sn) | oz)};
}

// a * W_128^j for a compile-time j; exact for multiples of 32.
__device__ __forceinline__ pf2 pw128(pf2 a, int j, int oz = 0) {
  j &= 127;
  if (j == 0) return a;
  if (j == 32) return pmi(a);
  if (j == 64) return -a;
  if (j == 96) return -pmi(a);
  return pcmul(a, w128(j, oz));
}

__device__ __forceinline__ void pdft4(pf2& a0, pf2& a1, pf2& a2, pf2& a3) {
  const pf2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, d = a1 - a3;
  a0 = t0 + t2;
  a1 = vadd_mi(t1, d);
  a2 = t0 - t2;
  a3 = vsub_mi(t1, d);
}

// In-place 16- and 32-point DFTs, natural order in and out (dft<16>'s 4 x 4
// split; 32 = 2 x 16 with a radix-2 combine).
__device__ __forceinline__ void pdft16(pf2 (&v)[16], int oz = 0) {
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) pdft4(v[n2], v[4 + n2], v[8 + n2], v[12 + n2]);
#pragma unroll
  for (int k1 = 1; k1 < 4; ++k1)
#pragma unroll
    for (int n2 = 1; n2 < 4; ++n2) v[4 * k1 + n2] = pw128(v[4 * k1 + n2], 8 * n2 * k1, oz);
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) pdft4(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
  pf2 o[16];
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) o[k1 + 4 * k2] = v[4 * k1 + k2];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = o[i];
}

__device__ __forceinline__ void pdft32(pf2 (&v)[32], int oz = 0) {
  pf2 e[16], o[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    e[i] = v[2 * i];
    o[i] = v[2 * i + 1];
  }
  pdft16(e, oz);
  pdft16(o, oz);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const pf2 t = pw128(o[k], 4 * k, oz);
    v[k] = e[k] + t;
    v[k + 16] = e[k] - t;
  }
}

// Orders this wave's LDS accesses (they execute in order within a wave; this
// keeps the compiler from moving them across the exchange).
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float swap_pair(float v) {  // the value of lane L ^ 1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}
__device__ __forceinline__ float bperm(int addr, float v) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v)));
}

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// Frame t's samples, lane's pairs (x[128 n1 + 2 lane], x[128 n1 + 2 lane + 1]),
// through a raw buffer resource over the frame: samples past the frame's valid
// range read as zeros (the zero padding of dsp_core.py:81-82).
__device__ __forceinline__ void wave_frame_load(const FftArgs& a, int64_t t, int lane,
                                                u32x2_t (&raw)[32]) {
  constexpr int N = 4096;
  const InRow ir = in_row<kSpec>(a, t);
  const int64_t valid = ir.valid < N ? (ir.valid > 0 ? ir.valid : 0) : N;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.in) + ir.base, 0, (int)(valid * 4), 0x00020000);
#pragma unroll
  for (int n1 = 0; n1 < 32; ++n1)
    raw[n1] = __builtin_amdgcn_raw_buffer_load_b64(rs, 8 * lane, 512 * n1, 2);
}

// The lane's index in its wave, recomputed (mbcnt) and opaque: a fresh copy
// per use site instead of one register live through the whole loop.
__device__ __forceinline__ int lane_now() {
  int l = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  asm volatile("" : "+v"(l));
  return l;
}

// One 4096-point transform t of the wave: raw = its frame's sample pairs
// (wave_frame_load), wl0 = the window in LDS, buf = the wave's transpose
// buffer.  Lane-derived values are recomputed (lane_now) in each phase
// instead of held through it: 4 waves per SIMD need <= 128 VGPRs.
__device__ __forceinline__ void w12_transform(const FftArgs& a, int64_t t, const u32x2_t (&raw)[32],
                                              const pf2* wl0, float* buf) {
  constexpr int N = 4096, NH = 2048;
  // (and of the window and twiddle addresses: hoisted, the window's 32 LDS
  // reads hold 64 VGPRs and the twiddles ~20)
  int z0 = 0;
  asm volatile("" : "+s"(z0));
  const pf2* win = wl0 + z0;
  pf2 v[32];
  const int l1 = lane_now();
  // (the window's LDS reads in groups of 8: all 32 in flight would hold 64
  // VGPRs beside the samples)
#pragma unroll
  for (int n1 = 0; n1 < 32; ++n1) {
    if (n1 % 8 == 0) asm volatile("" ::: "memory");
    v[n1] = pf2{__uint_as_float(raw[n1][0]), __uint_as_float(raw[n1][1])} * win[64 * n1 + l1];
  }
  // A: DFT over n1, then W_2048^(lane k1) / 2 (W_2048^m = W_4096^(2m); the
  // powers come from the table every 8 steps and by products in between)
  pdft32(v, z0);
  {
    // the step's twiddles, loaded only now (live through the DFT above
    // they cost ~10 VGPRs at its peak)
    int z1 = 0;
    asm volatile("" : "+s"(z1));
    const pf2* twp = reinterpret_cast<const pf2*>(a.tw) + z1;
    const int l2 = lane_now();
    const pf2 wl = twp[2 * l2];               // W_2048^lane
    pf2 w8[3];                                // W_2048^(8 lane k) / 2, k = 1..3
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const int m = (16 * l2 * k) & (N - 1);
      w8[k - 1] = (m < NH ? 0.5f : -0.5f) * twp[m & (NH - 1)];
    }
    pf2 p = 0.5f * wl;
    v[0] *= 0.5f;
#pragma unroll
    for (int k = 1; k < 32; ++k) {
      if (k % 8 == 0) {
        p = w8[k / 8 - 1];
      } else if (k > 1) {
        p = vcmul(p, wl);
      }
      v[k] = vcmul(v[k], p);
    }
  }
  // T: Y[k1][n2] -> lane 2 k1 + h reads Y[k1][2m + h], one plane at a time
  const int l3 = lane_now();
  const int rd = (l3 >> 1) * kWaveRow + (l3 & 1);  // transpose read base
  wave_lds_order();
#pragma unroll
  for (int k = 0; k < 32; ++k) buf[k * kWaveRow + l3] = v[k].x;
  wave_lds_order();
#pragma unroll
  for (int m = 0; m < 32; ++m) v[m].x = buf[rd + 2 * m];
  wave_lds_order();
#pragma unroll
  for (int k = 0; k < 32; ++k) buf[k * kWaveRow + l3] = v[k].y;
  wave_lds_order();
#pragma unroll
  for (int m = 0; m < 32; ++m) v[m].y = buf[rd + 2 * m];
  // B: DFT over m, then the radix-2 step across the lane pair: lane h = 1
  // scales its F_1 by W_64^j, the pair swaps, and Z = own * (+-1) + other
  pdft32(v, z0);
  const int l4 = lane_now();
  // (the lane's parity as an opaque float: the combine's 31 per-lane
  // twiddles are loop-invariant, and hoisting them would hold 62 VGPRs)
  const float hf = (float)(l4 & 1);
  const pf2 hh = pf2{hf, hf};
  const float sg = (l4 & 1) ? -1.f : 1.f;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    pf2 u = v[j];
    if (j > 0) {
      const pf2 one = pf2{1.f, 0.f};
      u = vcmul(u, one + hh * (w128(2 * j, z0) - one));  // h ? W_64^j : 1
    }
    v[j] = u * sg + pf2{swap_pair(u.x), swap_pair(u.y)};
  }
  // real split and |X[K]|; W_4096^K = W_4096^K0 W_128^j
  int z2 = 0;
  asm volatile("" : "+s"(z2));
  const int l5 = lane_now();
  const int src = ((1 - l5) & 63) << 2;     // bpermute address of Z[-K]'s lane
  const int K0 = (l5 >> 1) + 1024 * (l5 & 1);
  const pf2 wb = (reinterpret_cast<const pf2*>(a.tw) + z2)[K0];  // W_4096^K0
  float* mr = a.out + t * a.ld_out;
  pf2 prev = v[0];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const pf2 q = pf2{bperm(src, v[31 - j].x), bperm(src, v[31 - j].y)};
    const pf2 zm = l5 < 2 ? prev : q;
    prev = q;
    const pf2 zk = v[j];
    const pf2 sm = pf2{zk.x + zm.x, zk.y - zm.y};
    const pf2 d = pf2{zk.x - zm.x, zk.y + zm.y};
    const pf2 x = vcfma(d, pw128(wb, j + 32, z0), sm);  // s - i W d  (-i W_128^j = W_128^(j+32))
    mr[K0 + 32 * j] = cabsf_(make_float2(x.x, x.y));
  }
  if (l5 == 0) mr[NH] = 2.f * fabsf(v[0].x - v[0].y);  // X[N/2] = Re Z[0] - Im Z[0]
}

// A workgroup is a whole CU's 16 waves sharing one LDS copy of the window
// (16 KB + 16 transpose buffers = 151 KB), 4 waves per SIMD at <= 128 VGPRs
// (lane-derived values recomputed per phase, twiddles loaded where used; 4
// VGPRs spill, 20 B per lane); round 3's 4-wave groups held the LDS to 3
// groups = 3 waves per SIMD: 0.190 vs 0.1955 ms at config 4, 0.0295 vs 0.030
// at config 3 (profiles/r04_spec_ab.txt).  Measured and not adopted: the next
// frame in flight in 64 more VGPRs (2 waves per SIMD): 0.211 vs 0.193 ms at
// config 4 (round 3: 0.199 vs 0.194; profiles/r05_spec_pf_ab.txt); the waves
// of a SIMD starting 0.25 .. 1.5 us apart (round 5) or 4 .. 12 us apart (round
// 4): neutral / slower.  The memory-only floor of this launch (frame loads
// and |X| stores, no transform) is 0.166 ms at config 4 and 22.6 us at config
// 3, against 0.194 / 0.0305 ms with the transform (profiles/r05_spec_floor.txt).
__global__ __launch_bounds__(64 * kWavePerGroup) void k_spec_wave12(FftArgs a) {
  constexpr int N = 4096;
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the window, once per workgroup (LDS latency instead of an L2 round trip
  // per transform), then one transpose buffer per wave
  for (int i = threadIdx.x; i < N / 4; i += 64 * kWavePerGroup)
    reinterpret_cast<f32x4_t*>(ldsf)[i] = reinterpret_cast<const f32x4_t*>(a.win)[i];
  __syncthreads();
  const pf2* wl0 = reinterpret_cast<const pf2*>(ldsf);
  float* buf = ldsf + N + wv * kWaveLds;
  const int64_t nw = (int64_t)gridDim.x * kWavePerGroup;
  u32x2_t raw[32];
  for (int64_t t = (int64_t)blockIdx.x * kWavePerGroup + wv; t < a.B; t += nw) {
    wave_frame_load(a, t, lane_now(), raw);
    w12_transform(a, t, raw, wl0, buf);
  }
}

int launch_spec_wave12(const FftArgs& a, hipStream_t s) {
  const size_t shm = (size_t)(4096 + kWavePerGroup * kWaveLds) * sizeof(float);
  if (int rc = allow_lds(k_spec_wave12, shm)) return rc;
  const int res = resident_groups<k_spec_wave12>(64 * kWavePerGroup, shm);
  DSP_REQUIRE(res > 0, "occupancy query failed");
  const int64_t groups = ceil_div(a.B, kWavePerGroup);
  const unsigned grid = (unsigned)(groups < res ? groups : res);
  hipLaunchKernelGGL(k_spec_wave12, dim3(grid), dim3(64 * kWavePerGroup), shm, s, a);
  DSP_LAUNCHED("k_spec_wave12");
  return DSP_OK;
}

// ---------------------------------------------------------------------------
// Four-step FFT for N = 2^15 .. 2^DSP_MAX_LOG2N_FOURSTEP (beyond one workgroup's
// LDS): N = NA * NB, n = n1 + NB n2, k = k2 + NA k1 (n1, k1 < NB; n2, k2 < NA)
//   step A: Y[n1][k2] = W_N^(n1 k2) * sum_n2 x[n1 + NB n2] W_NA^(n2 k2)
//           -> workspace[k2][n1]
//   step B: X[k2 + NA k1] = sum_n1 Y[n1][k2] W_NB^(n1 k1)
// Each workgroup runs KC sub-transforms of consecutive columns (step A) or
// rows (step B) in LDS with the one-launch Stockham passes; the HBM side of
// both steps moves KC consecutive complex values per index (8 -- 64 B -- or
// 16 for the three-pass split's megabyte-strided passes), staged through LDS
// so that every global access is a run of consecutive addresses.  Up to 2^22
// two launches (sub-transforms up to 2^11); from 2^23 step B is itself a
// four-step (run_fft6_row).  The sub-transforms' twiddles come from the
// caller's W_N table at stride N/NA (N/NB), the inter-step twiddle W_N^m from
// the same table (m < N/2, else its negation), above 2^20 points as the
// product of two factors from small contiguous tables (tw_fetch).  The
// workspace holds Y: B x N complex (two launches) or Y, Y': 2 x N (three).
// ---------------------------------------------------------------------------
constexpr int kCols = 8;
// Columns per workgroup for a sub-transform of 2^LOG2 points: KC images of
// (N + N/16 + 1) complex values within 160 KB of LDS.
__host__ __device__ constexpr int kcols_for(int log2) {
  return log2 <= 11 ? kCols : log2 == 12 ? 4 : log2 == 13 ? 2 : 1;
}

struct Fft4Args {
  FftArgs a;          // in / out / rows / segment / window / W_N table
  float2* ws;         // B x N complex
  int64_t N;          // NA * NB
  uint32_t* hdr;      // per row: non-finite flag, list length (fft_nf.hip); NULL: none
  int64_t tws = 1;    // a.tw is the table of N * tws points (nested inner steps)
  int64_t nest = 0;   // step B of a nested inner transform: the outer NA (run_fft6_row)
  const float2* twc = nullptr;  // N * tws > 2^20: W^(i << tsh), i < (N * tws) >> tsh
  int tsh = 0;
};

// The inter-step twiddle W_Nt^m, Nt = N * tws.  Up to 2^20 points one read of
// the caller's table; above, W^m = W^(hi << tsh) W^lo with lo < 2^tsh, tsh =
// ceil(log2 Nt / 2): the fine factor from the table's first 2^tsh entries, the
// coarse one from the 2^(log2 Nt - tsh) entries k_tw_coarse gathered into the
// workspace -- both contiguous and L2-resident, where the workgroup's W^(n1 k2)
// alone are scattered over the whole table (one line fetched per 8-byte
// twiddle: round 5 measured the 2^28 four-step at 0.49 TB/s).  One more
// rounding (~1 ulp of 1), far inside the FFT's 1e-5.  In two halves, so that
// the table loads can be issued long before the value is needed (a select or
// product on the loaded values would make the compiler wait for them at
// once): w = sgn * a * b.
struct TwLoad {
  float2 a, b;
  float sgn;
};
__device__ __forceinline__ TwLoad tw_fetch(const Fft4Args& f, int64_t m) {
  // branch-free (a branch would join the loaded values through copies, which
  // wait for them): without the coarse table b is the table's W^0 = 1
  const int64_t Nt = f.N * f.tws;
  m &= Nt - 1;
  const bool split = f.twc != nullptr, up = !split && m >= Nt / 2;
  const float2* pa = split ? f.twc : f.a.tw;
  const int64_t ia = split ? m >> f.tsh : (up ? m - Nt / 2 : m);
  const int64_t ib = split ? m & ((int64_t(1) << f.tsh) - 1) : 0;
  return TwLoad{pa[ia], f.a.tw[ib], up ? -1.f : 1.f};
}
__device__ __forceinline__ float2 tw_finish(const TwLoad& t) {
  const float2 w = make_float2(t.a.x * t.b.x - t.a.y * t.b.y, t.a.x * t.b.y + t.a.y * t.b.x);
  return make_float2(t.sgn * w.x, t.sgn * w.y);
}

__global__ __launch_bounds__(256) void k_tw_coarse(const float2* __restrict__ tw, float2* twc,
                                                   int64_t N, int tsh) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < (N >> tsh)) twc[i] = tw_full(tw, i << tsh, N);
}

// Four-step sizes whose twiddles go through the coarse table, its shift and
// its size in bytes.
constexpr int kLog2TwSplit = 20;
inline int tw_shift(int log2n) { return (log2n + 1) / 2; }
inline size_t tw_coarse_bytes(int log2n) {
  return log2n > kLog2TwSplit ? (size_t(1) << (log2n - tw_shift(log2n))) * sizeof(float2) : 0;
}
int build_tw_coarse(const float2* tw, float2* twc, int log2n, hipStream_t s) {
  const int64_t n = int64_t(1) << (log2n - tw_shift(log2n));
  hipLaunchKernelGGL(k_tw_coarse, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, tw, twc,
                     int64_t(1) << log2n, tw_shift(log2n));
  DSP_LAUNCHED("k_tw_coarse");
  return DSP_OK;
}

// Step A's input (f.hdr set): a non-finite value raises the row's flag for the
// non-finite repair (fft_nf.hip) and, for the complex transforms, reads as
// zero, so that the output holds the DFT of the finite part -- the values the
// reference gives the components that no inf or NaN reaches.  (The spectrum's
// bins all become +inf or NaN; the repair rewrites every one.)
template <int LOG2A, int MODE, int KC = kcols_for(LOG2A)>
__global__ __launch_bounds__(KC * Plan<LOG2A>::TPT) void k_fft4_a(Fft4Args f) {
  using PL = Plan<LOG2A>;
  constexpr int NA = PL::N, NT = KC * PL::TPT, TS = PL::PADN + 1;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  const FftArgs& a = f.a;
  const int64_t NB = f.N / NA;
  const int64_t b = blockIdx.y;
  // XCD-aware: the workgroups the dispatcher sends to one XCD (every 8th) take
  // consecutive column groups, so the two 64-byte halves of a 128-byte line
  // are fetched into the same L2
  int64_t gx = blockIdx.x;
  if ((gridDim.x & 7) == 0) gx = (gx & 7) * (gridDim.x >> 3) + (gx >> 3);
  const int64_t c0 = gx * KC;
  const InRow ir = in_row<MODE>(a, b);
  // every load of the tile issued before the first use (PER per thread, in
  // registers), then the non-finite scan, then LDS: a loop that stored each
  // value as it arrived waited out one HBM round trip per value (round 5)
  constexpr int PER = KC * NA / NT;
  static_assert(PER * NT == KC * NA, "tile split");
  float2 v[PER];
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const int i = threadIdx.x + it * NT;
    v[it] = load_input<MODE>(a, ir, (int)(c0 + i % KC + NB * (i / KC)), true);
  }
  if (f.hdr) {
    // (the spectrum only flags: s * w is non-finite exactly when the sample s
    // is, w in [0, 1])
    bool nf = false;
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      if (!__builtin_isfinite(v[it].x)) {
        nf = true;
        if constexpr (MODE != kSpec) v[it].x = 0.f;
      }
      if constexpr (MODE != kSpec) {
        if (!__builtin_isfinite(v[it].y)) {
          nf = true;
          v[it].y = 0.f;
        }
      }
    }
    if (nf) f.hdr[2 * b] = 1u;
  }
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const int i = threadIdx.x + it * NT;
    lds[(i % KC) * TS + lpad(i / KC)] = v[it];
  }
  const int tl = threadIdx.x / PL::TPT, j0 = threadIdx.x - tl * PL::TPT;
  Tw<LOG2A, 0> tw;
  load_tw<LOG2A, 0>(tw, a.tw, j0, f.N / NA * f.tws);
  // The inter-step twiddles W_Nt^(n1 k2) of this thread's outputs: its column
  // n1 is fixed and k2 = r0 + it S, so three table values -- W^(n1 r0),
  // W^(n1 S), W^(4 n1 S) -- and products: W^(n1 (r0 + 4 q S)) by q - 1
  // multiplications by W^(4 n1 S), then W^(n1 S j), j = 1..3 (at most 6
  // roundings more than the table, ~4e-7; the passes' own twiddles chain up
  // to 15).  Their loads go out here, behind the passes' twiddles, so that
  // they are in flight under the passes (the barriers below wait for LDS
  // only).  Round 5: the epilogue loaded them itself, 4 outputs at a time --
  // 4 table round trips per tile, which held step A at ~2.1 TB/s against step
  // B's 4.6; fetched here as 4 anchors + W^(n1 S), 2^28 4.43 -> 3.55 ms; as
  // these 3, 3.38 ms (fewer scattered table reads).
  constexpr int S = NT / KC;
  static_assert(PER % 4 == 0 && NT % KC == 0, "twiddle anchors");
  const int c = threadIdx.x % KC, r0 = threadIdx.x / KC;
  const int64_t n1 = c0 + c;
  const TwLoad a0_l = tw_fetch(f, n1 * r0 * f.tws);
  const TwLoad s4_l = tw_fetch(f, n1 * 4 * S * f.tws);
  const TwLoad s1_l = tw_fetch(f, n1 * S * f.tws);
  lds_barrier();
  run_pass<LOG2A, 0>(LdsIO<NA>{lds + tl * TS}, lds + tl * TS, j0, tw);
  lds_barrier();
  const float2 s1 = tw_finish(s1_l), s2 = cmul(s1, s1), s3 = cmul(s2, s1), s4 = tw_finish(s4_l);
  float2 anc[PER / 4];
  anc[0] = tw_finish(a0_l);
#pragma unroll
  for (int q = 1; q < PER / 4; ++q) anc[q] = cmul(anc[q - 1], s4);
  float2* y = f.ws + b * f.N;
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const int k2 = r0 + it * S;
    const float2 w0 = anc[it / 4];
    const float2 w = it % 4 == 0 ? w0 : cmul(w0, it % 4 == 1 ? s1 : it % 4 == 2 ? s2 : s3);
    y[(int64_t)k2 * NB + n1] = cmul(lds[c * TS + lpad(k2)], w);
  }
}

// Step B.  Nested (run_fft6_row, f.nest = the outer NA): the KC rows of a
// workgroup are one inner row r = blockIdx.y of KC consecutive outer rows k2 =
// blockIdx.x KC + c, so that the natural-order output k of (k2, r), X[k2 +
// nest k], is written in runs of KC consecutive addresses, and the workgroups
// that write the other halves of those lines are dispatched to the same XCD
// at the same time (blockIdx.x remapped as in step A).
template <int LOG2B, int MODE, int KC = kcols_for(LOG2B)>
__global__ __launch_bounds__(KC * Plan<LOG2B>::TPT) void k_fft4_b(Fft4Args f) {
  using PL = Plan<LOG2B>;
  constexpr int NB = PL::N, NT = KC * PL::TPT, TS = PL::PADN + 1;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  const FftArgs& a = f.a;
  const int64_t NA = f.N / NB;
  // source row of lane group c: ws + src0 + c * src_c; output k1 of it at
  // out0 + c * out_c + k1 * out_k (complex / magnitude units)
  int64_t src0, src_c, out0, out_c, out_k;
  if (f.nest) {
    int64_t gx = blockIdx.x;
    if ((gridDim.x & 7) == 0) gx = (gx & 7) * (gridDim.x >> 3) + (gx >> 3);
    const int64_t k2 = gx * KC, r = blockIdx.y;
    src0 = k2 * f.N + r * NB;
    src_c = f.N;
    out0 = k2 + f.nest * r;
    out_c = 1;
    out_k = f.nest * NA;
  } else {
    const int64_t b = blockIdx.y, r0 = (int64_t)blockIdx.x * KC;  // first k2 row
    src0 = b * f.N + r0 * NB;
    src_c = NB;
    out0 = b * a.ld_out + r0;
    out_c = 1;
    out_k = NA;
  }
  const float2* y = f.ws + src0;
  constexpr int PER = KC * NB / NT;
  static_assert(PER * NT == KC * NB, "tile split");
  float2 v[PER];
#pragma unroll
  for (int it = 0; it < PER; ++it) {  // all loads in flight before the first LDS write
    const int i = threadIdx.x + it * NT;
    v[it] = y[(i / NB) * src_c + (i % NB)];
  }
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const int i = threadIdx.x + it * NT;
    lds[(i / NB) * TS + lpad(i % NB)] = v[it];
  }
  const int tl = threadIdx.x / PL::TPT, j0 = threadIdx.x - tl * PL::TPT;
  Tw<LOG2B, 0> tw;
  load_tw<LOG2B, 0>(tw, a.tw, j0, f.N / NB * f.tws);
  __syncthreads();
  run_pass<LOG2B, 0>(LdsIO<NB>{lds + tl * TS}, lds + tl * TS, j0, tw);
  __syncthreads();
  // the spectrum keeps k <= N_outer / 2 (row-relative index: out - row base)
  const int64_t onh = f.N * (f.nest ? f.nest : 1) / 2;
  const int64_t rel0 = f.nest ? out0 : out0 - (int64_t)blockIdx.y * a.ld_out;
  for (int i = threadIdx.x; i < KC * NB; i += NT) {
    const int c = i % KC, k1 = i / KC;
    const int64_t d = c * out_c + k1 * out_k;
    const float2 v = lds[c * TS + lpad(k1)];
    if constexpr (MODE == kSpec) {
      if (rel0 + d <= onh) a.out[out0 + d] = cabsf_(v);
    } else {
      reinterpret_cast<float2*>(a.out)[out0 + d] = v;
    }
  }
}

template <int LOG2A, int LOG2B, int MODE>
int launch_fft4(const Fft4Args& f, hipStream_t s) {
  using PA = Plan<LOG2A>;
  using PB = Plan<LOG2B>;
  static_assert(LOG2A >= 4 && LOG2B >= LOG2A, "split");
  // step A's columns 16 wide (128-byte runs) where two images fit a CU's LDS:
  // batched 2^15 .. 2^18, 3.5-4.1 -> 4.1-4.3 TB/s (round 5,
  // profiles/r05_fft_large.txt); step B reads whole rows either way
  constexpr int KA = LOG2A <= 9 ? 16 : kcols_for(LOG2A), KB = kcols_for(LOG2B);
  const size_t sa = (size_t)KA * (PA::PADN + 1) * sizeof(float2);
  const size_t sb = (size_t)KB * (PB::PADN + 1) * sizeof(float2);
  if (int rc = allow_lds(k_fft4_a<LOG2A, MODE, KA>, sa)) return rc;
  if (int rc = allow_lds(k_fft4_b<LOG2B, MODE>, sb)) return rc;
  const unsigned rows = (unsigned)f.a.B;
  hipLaunchKernelGGL((k_fft4_a<LOG2A, MODE, KA>), dim3((unsigned)(PB::N / KA), rows),
                     dim3(KA * PA::TPT), sa, s, f);
  DSP_LAUNCHED("k_fft4_a");
  hipLaunchKernelGGL((k_fft4_b<LOG2B, MODE>), dim3((unsigned)(PA::N / KB), rows),
                     dim3(KB * PB::TPT), sb, s, f);
  DSP_LAUNCHED("k_fft4_b");
  return DSP_OK;
}

template <int MODE>
int dispatch4(const Fft4Args& f, int log2n, hipStream_t s) {
  switch (log2n) {
    case 15: return launch_fft4<7, 8, MODE>(f, s);
    case 16: return launch_fft4<8, 8, MODE>(f, s);
    case 17: return launch_fft4<8, 9, MODE>(f, s);
    case 18: return launch_fft4<9, 9, MODE>(f, s);
    case 19: return launch_fft4<9, 10, MODE>(f, s);
    case 20: return launch_fft4<10, 10, MODE>(f, s);
    case 21: return launch_fft4<10, 11, MODE>(f, s);
    case 22: return launch_fft4<11, 11, MODE>(f, s);  // (2^23 and up: run_fft6_row)
    default: return set_error(DSP_EINVAL, "log2n=%d outside [0, %d]", log2n, DSP_MAX_LOG2N_FOURSTEP);
  }
}

// Three-pass (nested) four-step from N = 2^23 up to 2^30 (round 5; the
// reference's recursion has no size limit, dsp_core.py:41-66): N = NA * NB
// with NB = NB1 * NB2, so that no sub-transform exceeds 2^11 points and every
// HBM access is a run of 8 or 16 consecutive complex values (the two-step
// split of 2^24 and up needs sub-transforms of 2^12..2^14, 4..1 columns):
//   step A   (k_fft4_a<LA>): the NB columns of NA points of the row, the
//            twiddle W_N^(n1 k2) on the way out -> Y[k2][n1] (rows of NB);
//   step A'  (k_fft4_a<LA1>, complex): the NA rows' columns of NB1 points
//            with W_NB = W_N^NA (table stride tws = NA) -> Y'[k2][..];
//   step B'  (k_fft4_b<LB2>, nest = NA): rows of NB2 points, 8 or 16 outer
//            rows k2 per workgroup, natural-order output k of row k2 ->
//            X[k2 + NA k].
// Steps A and B' touch HBM at megabyte strides, A' at kilobyte ones.  One row
// at a time (the workspace is 2 N complex whatever B).  From 2^23: the
// two-pass split's 2^12..2^14-point sub-transforms move 4..1 columns per
// access; with the twiddle loads under the passes (k_fft4_a) round 5 measured
// 0.092 vs 0.111 ms at 2^23, 0.211 vs 0.274 at 2^24 and the two-pass faster at
// 2^22, 0.052 vs 0.057 ms (profiles/r05_fft_large.txt).
constexpr int kLog2Nested = 23;
static_assert(kLog2Nested > DSP_MAX_LOG2N + 1 && kLog2Nested <= DSP_MAX_LOG2N_FOURSTEP, "nest from");

template <int LA, int LA1, int LB2, int MODE>
int run_fft6_row(const FftArgs& row, float2* Y, float2* Y2, const float2* twc, uint32_t* hdr,
                 hipStream_t s) {
  constexpr int64_t N = int64_t(1) << (LA + LA1 + LB2);
  constexpr int64_t NA = int64_t(1) << LA, NB = N / NA;
  // 16 columns (128-byte runs) for the two passes whose HBM side is strided
  // by megabytes where the LDS image fits twice per CU (up to 2^9 points):
  // tools/stride_probe.hip copies such columns at 4.4 TB/s in 128-byte runs,
  // 2.9 in 64-byte runs; the middle pass (kilobyte strides, 5.0) keeps 8
  constexpr int KA = LA <= 9 ? 16 : kCols, K1 = kcols_for(LA1);
  constexpr int KB = LB2 <= 9 ? 16 : kCols;
  static_assert(NA % KB == 0 && (NB >> LA1) % K1 == 0, "3-pass split");
  using PA = Plan<LA>;
  using P1 = Plan<LA1>;
  using PB = Plan<LB2>;
  const size_t sa = (size_t)KA * (PA::PADN + 1) * sizeof(float2);
  const size_t s1 = (size_t)K1 * (P1::PADN + 1) * sizeof(float2);
  const size_t sb = (size_t)KB * (PB::PADN + 1) * sizeof(float2);
  if (int rc = allow_lds(k_fft4_a<LA, MODE, KA>, sa)) return rc;
  if (int rc = allow_lds(k_fft4_a<LA1, kC2C>, s1)) return rc;
  if (int rc = allow_lds(k_fft4_b<LB2, MODE, KB>, sb)) return rc;
  Fft4Args fa{row, Y, N, hdr};
  fa.twc = twc;
  fa.tsh = tw_shift(LA + LA1 + LB2);
  hipLaunchKernelGGL((k_fft4_a<LA, MODE, KA>), dim3((unsigned)(NB / KA), 1), dim3(KA * PA::TPT),
                     sa, s, fa);
  DSP_LAUNCHED("k_fft4_a");
  // the inner transforms over the NA rows of Y: complex in, W_NB from the W_N
  // table at stride NA
  const FftArgs inner{reinterpret_cast<const float*>(Y), row.out, NA, NB, row.ld_out, 0, 0, 0, 1,
                      nullptr, row.tw};
  Fft4Args f1{inner, Y2, NB, nullptr};
  f1.tws = NA;
  f1.twc = twc;
  f1.tsh = fa.tsh;
  hipLaunchKernelGGL((k_fft4_a<LA1, kC2C>), dim3((unsigned)((NB >> LA1) / K1), (unsigned)NA),
                     dim3(K1 * P1::TPT), s1, s, f1);
  DSP_LAUNCHED("k_fft4_a");
  Fft4Args fb = f1;
  fb.nest = NA;
  hipLaunchKernelGGL((k_fft4_b<LB2, MODE, KB>), dim3((unsigned)(NA / KB), (unsigned)(NB >> LB2)),
                     dim3(KB * PB::TPT), sb, s, fb);
  DSP_LAUNCHED("k_fft4_b");
  return DSP_OK;
}

template <int MODE>
int dispatch6(const FftArgs& row, int log2n, float2* Y, float2* Y2, const float2* twc,
              uint32_t* hdr, hipStream_t s) {
  switch (log2n) {
    case 23: return run_fft6_row<7, 8, 8, MODE>(row, Y, Y2, twc, hdr, s);
    case 24: return run_fft6_row<8, 8, 8, MODE>(row, Y, Y2, twc, hdr, s);
    // the strided passes (A, B') at most 2^9 where the split allows (16
    // columns, 128-byte runs), the middle one takes the rest; round 5 measured
    // 4.93 -> 4.46 ms at 2^28 against an even split with 8 columns, 2^30's
    // 9 / 11 / 10 at 20.1 vs 20.7 ms for 10 / 10 / 10 (profiles/r05_fft_large.txt)
    case 25: return run_fft6_row<8, 9, 8, MODE>(row, Y, Y2, twc, hdr, s);
    case 26: return run_fft6_row<9, 8, 9, MODE>(row, Y, Y2, twc, hdr, s);
    case 27: return run_fft6_row<9, 9, 9, MODE>(row, Y, Y2, twc, hdr, s);
    case 28: return run_fft6_row<9, 10, 9, MODE>(row, Y, Y2, twc, hdr, s);
    case 29: return run_fft6_row<9, 11, 9, MODE>(row, Y, Y2, twc, hdr, s);
    case 30: return run_fft6_row<9, 11, 10, MODE>(row, Y, Y2, twc, hdr, s);
    default: return set_error(DSP_EINVAL, "log2n=%d outside the three-pass range", log2n);
  }
}

template <int MODE>
int dispatch(const FftArgs& a, int log2n, hipStream_t s);

int dispatch_spec(const FftArgs& a, int log2n, hipStream_t s) {
  switch (log2n) {  // sizes whose first pass has radix < 16: the streaming kernel
    case 6: return launch_spec_stream<6>(a, s);
    case 7: return launch_spec_stream<7>(a, s);
    case 8: return launch_spec_stream<8>(a, s);
    case 10: return launch_spec_stream<10>(a, s);
    case 11: return launch_spec_stream<11>(a, s);
    case 12: return launch_spec_wave12(a, s);
    case 14: return launch_spec_stream<14>(a, s);
    default: break;
  }
  switch (log2n) {
    case 5: return launch_spec_real<5>(a, s);
    case 6: return launch_spec_real<6>(a, s);
    case 7: return launch_spec_real<7>(a, s);
    case 8: return launch_spec_real<8>(a, s);
    case 9: return launch_spec_real<9>(a, s);
    case 10: return launch_spec_real<10>(a, s);
    case 11: return launch_spec_real<11>(a, s);
    case 12: return launch_spec_real<12>(a, s);
    case 13: return launch_spec_real<13>(a, s);
    case 14: return launch_spec_real<14>(a, s);
    default: return dispatch<kSpec>(a, log2n, s);
  }
}

// ---------------------------------------------------------------------------
// Any-length DFT by Bluestein's chirp-z identity (for app.py:322-324, whose
// np.fft.fft segments have length int(1024 * L/M), e.g. 1114 = 2 * 557):
//   w[k] = exp(-i pi k^2 / n),  X[k] = w[k] * sum_j (x[j] w[j]) conj(w[k-j]),
// a circular convolution of length M = 2^m >= 2n - 1 done as two M-point
// Stockham transforms in one workgroup's LDS:
//   A = FFT(x w, zero-padded);  D = FFT(conj(A * Bf));  X[k] = w[k] conj(D[k])
// with Bf = FFT(b)/M, b[j] = b[M-j] = conj(w[j]) (j < n), from the host in
// float64 (rounded to float32).  The 1/M of the inverse transform is in Bf.
// ---------------------------------------------------------------------------
struct BluArgs {
  const float* in;   // real rows or interleaved complex rows
  float* out;        // interleaved complex rows, n values
  int64_t B, n, ld_in, ld_out;
  int real_in;
  const float2* chirp;  // w[k], k < n
  const float2* bf;     // FFT_M(b) / M
  const float2* tw;     // exp(-2 pi i k / M), k < M/2
};

template <int N>
struct BluStage1 {
  static constexpr bool kLdsIn = false;
  const BluArgs& a;
  float2* buf;
  int64_t t;
  bool live;
  __device__ __forceinline__ float2 load(int j) const {
    if (!live || j >= a.n) return make_float2(0.f, 0.f);
    const float2 x = a.real_in ? make_float2(a.in[t * a.ld_in + j], 0.f)
                               : reinterpret_cast<const float2*>(a.in)[t * a.ld_in + j];
    return cmul(x, a.chirp[j]);
  }
  __device__ __forceinline__ void store(int k, float2 v) const {
    const float2 c = cmul(v, a.bf[k]);
    buf[lpad(k)] = make_float2(c.x, -c.y);
  }
};

template <int N>
struct BluStage2 {
  static constexpr bool kLdsIn = true;
  const BluArgs& a;
  float2* buf;
  int64_t t;
  bool live;
  __device__ __forceinline__ float2 load(int j) const { return buf[lpad(j)]; }
  __device__ __forceinline__ void store(int k, float2 v) const {
    if (live && k < a.n)
      reinterpret_cast<float2*>(a.out)[t * a.ld_out + k] =
          cmul(make_float2(v.x, -v.y), a.chirp[k]);
  }
};

template <int LOG2N>
__global__ __launch_bounds__(Plan<LOG2N>::NT) void k_bluestein(BluArgs a) {
  using PL = Plan<LOG2N>;
  static_assert(PL::NP >= 1, "Bluestein needs M >= 2");
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  const int tl = threadIdx.x / PL::TPT;
  const int j0 = threadIdx.x - tl * PL::TPT;
  const int64_t t = (int64_t)blockIdx.x * PL::TPB + tl;
  const bool live = t < a.B;
  float2* buf = lds + tl * PL::PADN;
  Tw<LOG2N, 0> tw;
  load_tw<LOG2N, 0>(tw, a.tw, j0);
  run_pass<LOG2N, 0>(BluStage1<PL::N>{a, buf, t, live}, buf, j0, tw);
  __syncthreads();  // stage 1's last pass wrote LDS
  run_pass<LOG2N, 0>(BluStage2<PL::N>{a, buf, t, live}, buf, j0, tw);
}

template <int LOG2N>
int launch_blu(const BluArgs& a, hipStream_t s) {
  using PL = Plan<LOG2N>;
  const size_t shm = (size_t)PL::TPB * PL::PADN * sizeof(float2);
  if (int rc = allow_lds(k_bluestein<LOG2N>, shm)) return rc;
  const unsigned grid = (unsigned)ceil_div(a.B, PL::TPB);
  hipLaunchKernelGGL(k_bluestein<LOG2N>, dim3(grid), dim3(PL::NT), shm, s, a);
  DSP_LAUNCHED("k_bluestein");
  return DSP_OK;
}

template <int MODE, int LOG2N>
int launch_one(const FftArgs& a, hipStream_t s) {
  using PL = Plan<LOG2N>;
  const size_t shm = (size_t)PL::TPB * PL::PADN * sizeof(float2);
  if (int rc = allow_lds(k_fft<LOG2N, MODE>, shm)) return rc;
  const unsigned grid = (unsigned)ceil_div(a.B, PL::TPB);
  hipLaunchKernelGGL((k_fft<LOG2N, MODE>), dim3(grid), dim3(PL::NT), shm, s, a);
  DSP_LAUNCHED("k_fft");
  return DSP_OK;
}

template <int MODE>
int dispatch(const FftArgs& a, int log2n, hipStream_t s) {
  switch (log2n) {
    case 0: return launch_one<MODE, 0>(a, s);
    case 1: return launch_one<MODE, 1>(a, s);
    case 2: return launch_one<MODE, 2>(a, s);
    case 3: return launch_one<MODE, 3>(a, s);
    case 4: return launch_one<MODE, 4>(a, s);
    case 5: return launch_one<MODE, 5>(a, s);
    case 6: return launch_one<MODE, 6>(a, s);
    case 7: return launch_one<MODE, 7>(a, s);
    case 8: return launch_one<MODE, 8>(a, s);
    case 9: return launch_one<MODE, 9>(a, s);
    case 10: return launch_one<MODE, 10>(a, s);
    case 11: return launch_one<MODE, 11>(a, s);
    case 12: return launch_one<MODE, 12>(a, s);
    case 13: return launch_one<MODE, 13>(a, s);
    case 14: return launch_one<MODE, 14>(a, s);
    default: return set_error(DSP_EINVAL, "log2n=%d outside [0, %d]", log2n, DSP_MAX_LOG2N);
  }
}

}  // namespace

namespace {
constexpr int64_t kMaxRows4 = 65535;  // grid y extent of the four-step kernels
}  // namespace

// Two-pass sizes: [Y: B x N complex][coarse twiddles][non-finite header: 2
// words per row of a launch part].  Three-pass (run_fft6_row, one row at a
// time): [Y: N][Y': N complex][coarse twiddles][header: 2 words per row].
// The coarse twiddle table (tw_fetch) above 2^20 points: 2^floor(log2n / 2)
// complex.
size_t fourstep_workspace_bytes(int64_t B, int log2n) {
  if (B <= 0 || log2n <= DSP_MAX_LOG2N || log2n > DSP_MAX_LOG2N_FOURSTEP) return 0;
  const bool three = log2n >= kLog2Nested;
  const size_t rows = three ? (size_t)B : (size_t)(B < kMaxRows4 ? B : kMaxRows4);
  const size_t data = mul_sat(three ? 2 : (size_t)B, (size_t)1 << log2n, sizeof(float2));
  return add_sat(add_sat(data, tw_coarse_bytes(log2n)), mul_sat(rows, 2, sizeof(uint32_t)));
}

// The FFT's workspace (dsp_fft_workspace_bytes): the four-step's for one
// transform, the radix-2 split's (fft_split.hip) above it -- the larger of the
// two where a test hook (dsp_fft_split_log2n) sends four-step sizes through
// the split.
size_t fft_workspace_bytes(int64_t B, int log2n) {
  if (B <= 0 || log2n <= DSP_MAX_LOG2N || log2n > DSP_MAX_LOG2N_FFT) return 0;
  const size_t four = fourstep_workspace_bytes(B, log2n);
  const size_t split = fft_takes_split(log2n) ? fft_split_workspace_bytes(log2n) : 0;
  return four > split ? four : split;
}

namespace {

// Four-step transform of B rows, in launches of <= kMaxRows4 rows.
template <int MODE>
int run_fft4(FftArgs a, int log2n, void* ws, size_t ws_bytes, hipStream_t s) {
  DSP_REQUIRE(log2n <= DSP_MAX_LOG2N_FOURSTEP, "log2n=%d outside [0, %d]", log2n,
              DSP_MAX_LOG2N_FOURSTEP);
  const size_t need = fourstep_workspace_bytes(a.B, log2n);
  DSP_REQUIRE(ws && ws_bytes >= need, "FFT workspace too small: %zu < %zu bytes", ws_bytes, need);
  DSP_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 7) == 0, "FFT workspace not 8-byte aligned");
  const int64_t B = a.B;
  const int64_t N = int64_t(1) << log2n;
  if (log2n >= kLog2Nested) {
    float2* Y = static_cast<float2*>(ws);
    float2* twc = Y + 2 * N;
    uint32_t* hdr = reinterpret_cast<uint32_t*>(twc + tw_coarse_bytes(log2n) / sizeof(float2));
    if (int rc = build_tw_coarse(a.tw, twc, log2n, s)) return rc;
    DSP_HIP(hipMemsetAsync(hdr, 0, (size_t)B * 2 * sizeof(uint32_t), s));
    for (int64_t b = 0; b < B; ++b) {
      FftArgs row = a;
      row.B = 1;
      row.in = a.in + b * a.ld_in * (MODE == kC2C ? 2 : 1);
      row.out = a.out + b * a.ld_out * (MODE == kSpec ? 1 : 2);
      if (int rc = dispatch6<MODE>(row, log2n, Y, Y + N, twc, hdr + 2 * b, s)) return rc;
      const NfArgs nfa{row.in, row.out, 1, row.ld_in, row.ld_out, row.seg_start, row.seg_len,
                       row.hop, row.frames, row.win, reinterpret_cast<const float*>(row.tw), MODE,
                       log2n};
      if (int rc = launch_nf_large(nfa, hdr + 2 * b, reinterpret_cast<uint64_t*>(Y), N, s))
        return rc;
    }
    return DSP_OK;
  }
  float2* twc = tw_coarse_bytes(log2n) ? static_cast<float2*>(ws) + B * N : nullptr;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(static_cast<char*>(ws) + (size_t)B * N * 8 +
                                              tw_coarse_bytes(log2n));
  if (twc)
    if (int rc = build_tw_coarse(a.tw, twc, log2n, s)) return rc;
  for (int64_t b0 = 0; b0 < B; b0 += kMaxRows4) {
    FftArgs part = a;
    part.B = B - b0 < kMaxRows4 ? B - b0 : kMaxRows4;
    part.in = a.in + b0 * a.ld_in * (MODE == kC2C ? 2 : 1);
    part.out = a.out + b0 * a.ld_out * (MODE == kSpec ? 1 : 2);
    DSP_HIP(hipMemsetAsync(hdr, 0, (size_t)part.B * 2 * sizeof(uint32_t), s));
    Fft4Args f{part, static_cast<float2*>(ws), N, hdr};
    f.twc = twc;
    f.tsh = tw_shift(log2n);
    if (int rc = dispatch4<MODE>(f, log2n, s)) return rc;
    // the rows' non-finite inputs, listed in the freed Y rows
    const NfArgs nfa{part.in, part.out, part.B, part.ld_in, part.ld_out, part.seg_start,
                     part.seg_len, part.hop, part.frames, part.win,
                     reinterpret_cast<const float*>(part.tw), MODE, log2n};
    if (int rc = launch_nf_large(nfa, hdr, static_cast<uint64_t*>(ws), N, s)) return rc;
  }
  return DSP_OK;
}
}  // namespace

int launch_spectrum(const float* x, float* mag, int64_t B, int64_t ld_x,
                    int64_t seg_start, int64_t seg_len, int log2n,
                    int64_t ld_mag, const float* window, const float* tw,
                    void* ws, size_t ws_bytes, hipStream_t s, bool repair) {
  if (log2n > DSP_MAX_LOG2N) {
    DSP_REQUIRE(log2n <= DSP_MAX_LOG2N_FOURSTEP, "log2n=%d outside [0, %d]", log2n,
                DSP_MAX_LOG2N_FOURSTEP);
    const int64_t N = int64_t(1) << log2n;
    DSP_REQUIRE(B >= 0 && seg_start >= 0 && seg_len >= 0 && seg_len <= N,
                "bad segment start=%lld len=%lld (N=%lld)", (long long)seg_start,
                (long long)seg_len, (long long)N);
    DSP_REQUIRE(ld_mag >= N / 2 + 1, "ld_mag too small");
    DSP_REQUIRE(ld_x >= seg_start + seg_len, "segment exceeds the row");
    if (B == 0) return DSP_OK;
    DSP_REQUIRE(x && mag && window && tw, "null pointer");
    FftArgs a{x, mag, B, ld_x, ld_mag, seg_start, seg_len, 0, 1, window,
              reinterpret_cast<const float2*>(tw)};
    TraceScope trace("spectrum", s);
    return run_fft4<kSpec>(a, log2n, ws, ws_bytes, s);
  }
  return launch_stft(x, mag, B, ld_x, seg_start, seg_len, 0, 1, log2n, ld_mag, window, tw, s,
                     repair);
}

int launch_stft(const float* x, float* mag, int64_t B, int64_t ld_x, int64_t seg_start,
                int64_t seg_len, int64_t hop, int64_t frames, int log2n, int64_t ld_mag,
                const float* window, const float* tw, hipStream_t s, bool repair) {
  DSP_REQUIRE(log2n >= 0 && log2n <= DSP_MAX_LOG2N, "log2n=%d outside [0, %d]", log2n,
              DSP_MAX_LOG2N);
  const int64_t N = int64_t(1) << log2n;
  DSP_REQUIRE(frames >= 1 && hop >= 0 && (frames == 1 || hop >= 1), "bad framing hop=%lld "
              "frames=%lld", (long long)hop, (long long)frames);
  DSP_REQUIRE(B >= 0 && seg_start >= 0 && seg_len >= 0 && (frames > 1 || seg_len <= N),
              "bad segment start=%lld len=%lld (N=%lld)", (long long)seg_start,
              (long long)seg_len, (long long)N);
  DSP_REQUIRE(ld_mag >= N / 2 + 1, "ld_mag too small");
  DSP_REQUIRE(ld_x >= seg_start + seg_len, "segment exceeds the row");
  if (B == 0) return DSP_OK;
  DSP_REQUIRE(x && mag && window && tw, "null pointer");
  DSP_REQUIRE(B <= INT64_MAX / frames, "too many frames");
  FftArgs a{x, mag, B * frames, ld_x, ld_mag, seg_start, seg_len, hop, frames, window,
            reinterpret_cast<const float2*>(tw)};
  {
    TraceScope trace(frames == 1 ? "spectrum" : "stft", s);
    if (int rc = dispatch_spec(a, log2n, s)) return rc;
  }
  if (!repair) return DSP_OK;
  TraceScope trace("spectrum_nf", s);
  return launch_nf_small(NfArgs{x, mag, B * frames, ld_x, ld_mag, seg_start, seg_len, hop, frames,
                                window, tw, kSpec, log2n},
                         s);
}

int launch_fft(const float* in, float* out, int64_t B, int log2n, int real_in,
               int64_t ld_in, int64_t ld_out, const float* tw, void* ws, size_t ws_bytes,
               hipStream_t s) {
  DSP_REQUIRE(log2n >= 0 && log2n <= DSP_MAX_LOG2N_FFT, "log2n=%d outside [0, %d]", log2n,
              DSP_MAX_LOG2N_FFT);
  const int64_t N = int64_t(1) << log2n;
  DSP_REQUIRE(B >= 0 && ld_in >= N && ld_out >= N, "bad sizes");
  if (B == 0) return DSP_OK;
  DSP_REQUIRE(in && out && tw, "null pointer");
  DSP_REQUIRE((reinterpret_cast<uintptr_t>(out) & 7) == 0 &&
                  (real_in || (reinterpret_cast<uintptr_t>(in) & 7) == 0),
              "complex buffers must be 8-byte aligned");
  if (fft_takes_split(log2n))  // above one four-step transform (fft_split.hip)
    return launch_fft_split(in, out, B, log2n, real_in, ld_in, ld_out, tw, ws, ws_bytes, s);
  FftArgs a{in, out, B, ld_in, ld_out, 0, 0, 0, 1, nullptr, reinterpret_cast<const float2*>(tw)};
  if (log2n > DSP_MAX_LOG2N) {
    TraceScope trace("fft", s);
    return real_in ? run_fft4<kR2C>(a, log2n, ws, ws_bytes, s)
                   : run_fft4<kC2C>(a, log2n, ws, ws_bytes, s);
  }
  {
    TraceScope trace("fft", s);
    if (int rc = real_in ? dispatch<kR2C>(a, log2n, s) : dispatch<kC2C>(a, log2n, s)) return rc;
  }
  TraceScope trace("fft_nf", s);
  return launch_nf_small(NfArgs{in, out, B, ld_in, ld_out, 0, 0, 0, 1, nullptr, tw,
                                real_in ? kR2C : kC2C, log2n},
                         s);
}

}  // namespace dsp

namespace dsp {

int bluestein_log2m(int64_t n) {
  int m = 1;
  while ((int64_t(1) << m) < 2 * n - 1) ++m;
  return m;
}

int launch_dft(const float* in, float* out, int64_t B, int64_t n, int real_in, int64_t ld_in,
               int64_t ld_out, const float* chirp, const float* chirp_fft, const float* tw_m,
               hipStream_t s) {
  DSP_REQUIRE(n >= 1 && n <= DSP_MAX_DFT, "n=%lld outside [1, %d]", (long long)n, DSP_MAX_DFT);
  DSP_REQUIRE(B >= 0 && ld_in >= n && ld_out >= n, "bad sizes");
  if (B == 0) return DSP_OK;
  DSP_REQUIRE(in && out && chirp && chirp_fft && tw_m, "null pointer");
  DSP_REQUIRE((reinterpret_cast<uintptr_t>(out) & 7) == 0 &&
                  (real_in || (reinterpret_cast<uintptr_t>(in) & 7) == 0),
              "complex buffers must be 8-byte aligned");
  BluArgs a{in, out, B, n, ld_in, ld_out, real_in, reinterpret_cast<const float2*>(chirp),
            reinterpret_cast<const float2*>(chirp_fft), reinterpret_cast<const float2*>(tw_m)};
  TraceScope trace("dft", s);
  switch (bluestein_log2m(n)) {
    case 1: return launch_blu<1>(a, s);
    case 2: return launch_blu<2>(a, s);
    case 3: return launch_blu<3>(a, s);
    case 4: return launch_blu<4>(a, s);
    case 5: return launch_blu<5>(a, s);
    case 6: return launch_blu<6>(a, s);
    case 7: return launch_blu<7>(a, s);
    case 8: return launch_blu<8>(a, s);
    case 9: return launch_blu<9>(a, s);
    case 10: return launch_blu<10>(a, s);
    case 11: return launch_blu<11>(a, s);
    case 12: return launch_blu<12>(a, s);
    case 13: return launch_blu<13>(a, s);
    case 14: return launch_blu<14>(a, s);
    default: return set_error(DSP_EINVAL, "no Bluestein size for n=%lld", (long long)n);
  }
}

}  // namespace dsp
