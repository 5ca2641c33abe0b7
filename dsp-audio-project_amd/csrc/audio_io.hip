// Audio I/O edges of the hot path, gfx950.
//
// Loader: reference modules/dsp_core.py:10-35 (cargar_senal_audio) reads the
// file with soundfile (float64, integers scaled by 2^-(bits-1), unsigned 8-bit
// offset by 128), averages the channels (x_n.mean(axis=1), float64), casts to
// float32 and divides by max|x| when that exceeds 1e-6.  Here the host parses
// the RIFF/WAVE header (dsp_wav_parse, no sample touched), the raw PCM bytes go
// to the GPU as they are (2 bytes per 16-bit sample instead of 8 for float64),
// and two kernels finish the job:
//   k_pcm_mono:   decode + channel mean in float64 (numpy's summation order),
//                 rounded to float32 -- bit-identical to the reference;
//   k_absmax:     per-row max|x| as an unsigned max over float bits (NaN sorts
//                 above +inf, so a NaN peak propagates like np.max);
//   k_scale:      x /= peak (IEEE float32 division) where peak > threshold.
// Playback: reference app.py:349-355 turns z into 16-bit PCM: nan_to_num,
// divide by max|z| if > 0, * 32767, astype(int16) (truncation), all float64.
// k_quantize16 does exactly that per row from the float32 z the chain wrote.
// Everything is HBM-streaming integer/byte work: coalesced loads, one pass.
#include <cfloat>
#include <cmath>
#include <cstring>

#include <type_traits>

#include "common.h"

namespace dsp {
namespace {

constexpr int kIoNT = 256;

// Byte k of a W-byte little-endian value stored little- or big-endian.
template <int W, bool BE>
__device__ __forceinline__ uint32_t byte_at(const uint8_t* __restrict__ p, int k) {
  return p[BE ? W - 1 - k : k];
}

// G.711 expansions to 16-bit linear PCM, as libsndfile's tables (and the
// classic Sun g711.c) give them: mu-law peaks at +-32124, A-law at +-32256.
__device__ __forceinline__ int ulaw_to_s16(uint32_t u) {
  u = ~u & 0xFFu;
  const int t = ((((int)(u & 0x0F)) << 3) + 0x84) << ((u >> 4) & 7);
  return (u & 0x80) ? (0x84 - t) : (t - 0x84);
}
__device__ __forceinline__ int alaw_to_s16(uint32_t a) {
  a ^= 0x55;
  int t = (int)(a & 0x0F) << 4;
  const int seg = (int)((a & 0x70) >> 4);
  if (seg == 0) t += 8;
  else t = (t + 0x108) << (seg - 1);
  return (a & 0x80) ? t : -t;
}

// Sample c of frame i as soundfile returns it (float64).  FMT: DSP_WAV_PCM /
// FLOAT / ALAW / ULAW; BE: big-endian samples (AIFF); S8: signed 8-bit PCM
// (AIFF; WAV's is unsigned with a 128 offset).
template <int FMT, int BITS, bool BE = false, bool S8 = false>
__device__ __forceinline__ double decode(const uint8_t* __restrict__ p) {
  constexpr int W = BITS / 8;
  if constexpr (FMT == DSP_WAV_ULAW) {
    return (double)ulaw_to_s16(p[0]) / 32768.0;
  } else if constexpr (FMT == DSP_WAV_ALAW) {
    return (double)alaw_to_s16(p[0]) / 32768.0;
  } else if constexpr (FMT == DSP_WAV_FLOAT) {
    if constexpr (BITS == 32) {
      uint32_t u = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) u |= byte_at<4, BE>(p, k) << (8 * k);
      return (double)__uint_as_float(u);
    } else {
      uint64_t u = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) u |= (uint64_t)byte_at<8, BE>(p, k) << (8 * k);
      return __longlong_as_double((long long)u);
    }
  } else if constexpr (BITS == 8) {
    return S8 ? (double)(int8_t)p[0] / 128.0 : ((double)p[0] - 128.0) / 128.0;
  } else if constexpr (BITS == 16) {
    const int16_t v = (int16_t)(byte_at<2, BE>(p, 0) | (byte_at<2, BE>(p, 1) << 8));
    return (double)v / 32768.0;
  } else if constexpr (BITS == 24) {
    int32_t v = (int32_t)(byte_at<3, BE>(p, 0) | (byte_at<3, BE>(p, 1) << 8) |
                          (byte_at<3, BE>(p, 2) << 16));
    v = (int32_t)((uint32_t)v << 8) >> 8;  // sign-extend
    return (double)v / 8388608.0;
  } else {
    static_assert(W == 4, "PCM widths 8/16/24/32");
    const int32_t v = (int32_t)(byte_at<4, BE>(p, 0) | (byte_at<4, BE>(p, 1) << 8) |
                                (byte_at<4, BE>(p, 2) << 16) | (byte_at<4, BE>(p, 3) << 24));
    return (double)v / 2147483648.0;
  }
}

// np.add.reduce over a contiguous axis of length ch, then / ch: a plain loop
// below 8 elements, numpy's 8-accumulator pairwise block up to 128.
template <int FMT, int BITS, bool BE, bool S8>
__device__ __forceinline__ double channel_mean(const uint8_t* __restrict__ f, int ch) {
  constexpr int W = BITS / 8;
  if (ch == 1) return decode<FMT, BITS, BE, S8>(f);
  double s;
  if (ch < 8) {
    s = decode<FMT, BITS, BE, S8>(f);
    for (int c = 1; c < ch; ++c) s += decode<FMT, BITS, BE, S8>(f + c * W);
  } else {
    double r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = decode<FMT, BITS, BE, S8>(f + k * W);
    int c = 8;
    for (; c + 8 <= ch; c += 8) {
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] += decode<FMT, BITS, BE, S8>(f + (c + k) * W);
    }
    s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; c < ch; ++c) s += decode<FMT, BITS, BE, S8>(f + c * W);
  }
  return s / (double)ch;
}

template <int FMT, int BITS, bool BE, bool S8>
__global__ __launch_bounds__(kIoNT) void k_pcm_mono(const uint8_t* __restrict__ pcm, int ch,
                                                   int64_t frames, int64_t ld_bytes,
                                                   float* __restrict__ out, int64_t ld_out) {
  const int64_t b = blockIdx.y;
  const uint8_t* row = pcm + b * ld_bytes;
  float* o = out + b * ld_out;
  const int64_t stride = (int64_t)gridDim.x * kIoNT;
  for (int64_t i = (int64_t)blockIdx.x * kIoNT + threadIdx.x; i < frames; i += stride)
    o[i] = (float)channel_mean<FMT, BITS, BE, S8>(row + i * (int64_t)ch * (BITS / 8), ch);
}

// Row max of |x| as float bits (all non-negative, so unsigned order is float
// order, with NaN above +inf).  NAN0: NaN counts as 0 (np.nan_to_num first).
template <bool NAN0>
__global__ __launch_bounds__(kIoNT) void k_absmax(const float* __restrict__ x, int64_t n,
                                                 int64_t ld, uint32_t* __restrict__ peak) {
  const int64_t b = blockIdx.y;
  const float* r = x + b * ld;
  uint32_t m = 0;
  const int64_t stride = (int64_t)gridDim.x * kIoNT;
  for (int64_t i = (int64_t)blockIdx.x * kIoNT + threadIdx.x; i < n; i += stride) {
    uint32_t u = __float_as_uint(r[i]) & 0x7fffffffu;
    if (NAN0 && u > 0x7f800000u) u = 0;
    m = max(m, u);
  }
  // wave reduction, then one atomic per wave
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(peak + b, m);
}

__global__ __launch_bounds__(kIoNT) void k_scale(float* __restrict__ x, int64_t n, int64_t ld,
                                                const uint32_t* __restrict__ peak,
                                                double threshold) {
  const int64_t b = blockIdx.y;
  const float pk = __uint_as_float(peak[b]);
  if (!((double)pk > threshold)) return;  // NaN peak: unchanged, as in the reference
  float* r = x + b * ld;
  const int64_t stride = (int64_t)gridDim.x * kIoNT;
  for (int64_t i = (int64_t)blockIdx.x * kIoNT + threadIdx.x; i < n; i += stride)
    r[i] = r[i] / pk;
}

// app.py:349-355 in z_final's own dtype: float64 (F32 = false, z_final came
// out of the SRC or the EQ) or float32 (F32 = true: SRC and EQ both bypassed,
// z_final is the loader's float32 array).  nan_to_num maps NaN to 0 and +-inf
// to +-(the dtype's max), so an infinite peak is that max too.
template <bool F32>
__global__ __launch_bounds__(kIoNT) void k_quantize16(const float* __restrict__ z, int64_t n,
                                                     int64_t ld_z, int16_t* __restrict__ out,
                                                     int64_t ld_out,
                                                     const uint32_t* __restrict__ peak) {
  typedef typename std::conditional<F32, float, double>::type real;
  const real big = F32 ? (real)FLT_MAX : (real)DBL_MAX;
  const int64_t b = blockIdx.y;
  const uint32_t pu = peak[b];
  const real pk = pu == 0x7f800000u ? big : (real)__uint_as_float(pu);
  const float* r = z + b * ld_z;
  int16_t* o = out + b * ld_out;
  const int64_t stride = (int64_t)gridDim.x * kIoNT;
  for (int64_t i = (int64_t)blockIdx.x * kIoNT + threadIdx.x; i < n; i += stride) {
    real v = (real)r[i];
    if (v != v) v = 0;
    else if (v == (real)INFINITY) v = big;
    else if (v == -(real)INFINITY) v = -big;
    if (pk > 0) v /= pk;
    o[i] = (int16_t)(int)(v * (real)32767);  // truncation toward zero, |v * 32767| <= 32767
  }
}

unsigned io_blocks(int64_t n) {
  const int64_t want = ceil_div(n, (int64_t)kIoNT * 4);  // ~4 elements per thread
  return (unsigned)(want < 1 ? 1 : (want > 2048 ? 2048 : want));
}

// Rows ride on the grid's y extent (<= 65535): larger batches launch in
// consecutive row ranges, f(b0, nb) once per range.
constexpr int64_t kMaxRowsY = 65535;
template <class F>
int for_row_ranges(int64_t B, F f) {
  for (int64_t b0 = 0; b0 < B; b0 += kMaxRowsY)
    if (int rc = f(b0, B - b0 < kMaxRowsY ? B - b0 : kMaxRowsY)) return rc;
  return DSP_OK;
}

int absmax(const float* x, int64_t B, int64_t n, int64_t ld, uint32_t* peak, bool nan0,
           hipStream_t s) {
  DSP_HIP(hipMemsetAsync(peak, 0, (size_t)B * sizeof(uint32_t), s));
  if (n == 0) return DSP_OK;
  return for_row_ranges(B, [&](int64_t b0, int64_t nb) {
    const dim3 grid(io_blocks(n), (unsigned)nb);
    if (nan0)
      hipLaunchKernelGGL(k_absmax<true>, grid, dim3(kIoNT), 0, s, x + b0 * ld, n, ld, peak + b0);
    else
      hipLaunchKernelGGL(k_absmax<false>, grid, dim3(kIoNT), 0, s, x + b0 * ld, n, ld, peak + b0);
    DSP_LAUNCHED("k_absmax");
    return DSP_OK;
  });
}

// ---- batched loader (dsp_pcm_batch_to_mono_f32): one decode launch over a
// table of per-row descriptors, one normalise launch.
//
// Launch 1, k_pcm_batch: block (bx, b) decodes + averages row b's frames
// [bx kIoNT, ...) grid-stride as k_pcm_mono does (the row's format picks the
// decoder: a block-uniform branch), writes zeros past the row's frames up to
// the batch width, and stores its max |x| (float bits, k_absmax's order) in
// its own slot of the block-maxima table -- every slot written, no
// initialisation, no atomics.  Launch 2, k_scale_batch: each block reduces
// its row's slots to the peak and divides the row's frames by it where
// (double)peak > threshold; block 0 stores the peak.
template <int FMT, int BITS, bool BE, bool S8>
__device__ __forceinline__ uint32_t pcm_batch_row(const uint8_t* __restrict__ row, int ch,
                                                  int64_t frames, int64_t width,
                                                  float* __restrict__ o) {
  uint32_t m = 0;
  const int64_t stride = (int64_t)gridDim.x * kIoNT;
  for (int64_t i = (int64_t)blockIdx.x * kIoNT + threadIdx.x; i < width; i += stride) {
    const float v = i < frames
                        ? (float)channel_mean<FMT, BITS, BE, S8>(row + i * (int64_t)ch * (BITS / 8), ch)
                        : 0.f;
    o[i] = v;
    m = max(m, __float_as_uint(v) & 0x7fffffffu);
  }
  return m;
}

// Block-wide unsigned max (kIoNT threads); the result in thread 0.
__device__ __forceinline__ uint32_t block_umax(uint32_t m, uint32_t* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    for (int w = 1; w < kIoNT / 64; ++w) m = max(m, red[w]);
  return m;
}

// (format, bits) of a descriptor as one key.
__host__ __device__ constexpr int pcm_key(int format, int bits) { return format | (bits << 16); }

__global__ __launch_bounds__(kIoNT) void k_pcm_batch(const uint8_t* __restrict__ pcm,
                                                    const dsp_pcm_row* __restrict__ rows,
                                                    int64_t b0, int64_t width,
                                                    float* __restrict__ out, int64_t ld_out,
                                                    uint32_t* __restrict__ blockmax) {
  __shared__ uint32_t red[kIoNT / 64];
  const int64_t b = b0 + blockIdx.y;
  const dsp_pcm_row r = rows[b];
  const uint8_t* row = pcm + r.offset;
  float* o = out + blockIdx.y * ld_out;
  uint32_t m = 0;
  switch (pcm_key(r.format, r.bits)) {
#define DSP_PCMB(F, BI, FLAGS)                                                               \
  case pcm_key((F) | (FLAGS), BI):                                                           \
    m = pcm_batch_row<F, BI, ((FLAGS) & DSP_AUDIO_BE) != 0, ((FLAGS) & DSP_AUDIO_S8) != 0>(  \
        row, r.channels, r.frames, width, o);                                                \
    break;
    DSP_PCMB(DSP_WAV_PCM, 8, 0)
    DSP_PCMB(DSP_WAV_PCM, 8, DSP_AUDIO_S8)
    DSP_PCMB(DSP_WAV_PCM, 8, DSP_AUDIO_S8 | DSP_AUDIO_BE)
    DSP_PCMB(DSP_WAV_PCM, 16, 0)
    DSP_PCMB(DSP_WAV_PCM, 24, 0)
    DSP_PCMB(DSP_WAV_PCM, 32, 0)
    DSP_PCMB(DSP_WAV_PCM, 16, DSP_AUDIO_BE)
    DSP_PCMB(DSP_WAV_PCM, 24, DSP_AUDIO_BE)
    DSP_PCMB(DSP_WAV_PCM, 32, DSP_AUDIO_BE)
    DSP_PCMB(DSP_WAV_FLOAT, 32, 0)
    DSP_PCMB(DSP_WAV_FLOAT, 64, 0)
    DSP_PCMB(DSP_WAV_FLOAT, 32, DSP_AUDIO_BE)
    DSP_PCMB(DSP_WAV_FLOAT, 64, DSP_AUDIO_BE)
    DSP_PCMB(DSP_WAV_ULAW, 8, 0)
    DSP_PCMB(DSP_WAV_ALAW, 8, 0)
    DSP_PCMB(DSP_WAV_ULAW, 8, DSP_AUDIO_BE)
    DSP_PCMB(DSP_WAV_ALAW, 8, DSP_AUDIO_BE)
#undef DSP_PCMB
    default:
      break;  // the host validated every descriptor
  }
  m = block_umax(m, red);
  if (threadIdx.x == 0) blockmax[b * gridDim.x + blockIdx.x] = m;
}

__global__ __launch_bounds__(kIoNT) void k_scale_batch(float* __restrict__ out, int64_t ld_out,
                                                      const dsp_pcm_row* __restrict__ rows,
                                                      int64_t b0, const uint32_t* __restrict__ blockmax,
                                                      int nbx, double threshold,
                                                      uint32_t* __restrict__ peak_out) {
  __shared__ uint32_t red[kIoNT / 64];
  __shared__ uint32_t pk_bits;
  const int64_t b = b0 + blockIdx.y;
  uint32_t m = 0;
  for (int i = threadIdx.x; i < nbx; i += kIoNT) m = max(m, blockmax[b * nbx + i]);
  m = block_umax(m, red);
  if (threadIdx.x == 0) {
    pk_bits = m;
    if (blockIdx.x == 0) peak_out[b] = m;
  }
  __syncthreads();
  const float pk = __uint_as_float(pk_bits);
  if (!((double)pk > threshold)) return;  // NaN peak: unchanged, as in the reference
  const int64_t frames = rows[b].frames;
  float* o = out + blockIdx.y * ld_out;
  const int64_t stride = (int64_t)gridDim.x * kIoNT;
  for (int64_t i = (int64_t)blockIdx.x * kIoNT + threadIdx.x; i < frames; i += stride)
    o[i] = o[i] / pk;
}

uint32_t rd32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
void wr32(uint8_t* p, uint32_t v) { for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i)); }
void wr16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }

}  // namespace

int wav_parse(const uint8_t* buf, size_t len, dsp_wav_info* info) {
  DSP_REQUIRE(buf && info, "null pointer");
  DSP_REQUIRE(len >= 12 && !memcmp(buf, "RIFF", 4) && !memcmp(buf + 8, "WAVE", 4),
              "not a RIFF/WAVE file");
  bool have_fmt = false;
  int tag = 0;
  dsp_wav_info w{};
  size_t pos = 12;
  while (pos + 8 <= len) {
    const uint32_t sz = rd32(buf + pos + 4);
    const uint8_t* body = buf + pos + 8;
    const size_t avail = len - (pos + 8);
    if (!memcmp(buf + pos, "fmt ", 4)) {
      DSP_REQUIRE(sz >= 16 && avail >= 16, "truncated fmt chunk");
      tag = rd16(body);
      w.channels = rd16(body + 2);
      w.sample_rate = (int32_t)rd32(body + 4);
      w.bits = rd16(body + 14);
      if (tag == 0xFFFE) {  // WAVE_FORMAT_EXTENSIBLE: the sub-format GUID starts with the tag
        DSP_REQUIRE(sz >= 40 && avail >= 26, "truncated extensible fmt chunk");
        tag = rd16(body + 24);
      }
      have_fmt = true;
    } else if (!memcmp(buf + pos, "data", 4)) {
      DSP_REQUIRE(have_fmt, "data chunk before fmt chunk");
      w.data_offset = (int64_t)(pos + 8);
      // A streamed header may carry a size past the end: read what is there.
      w.data_bytes = (int64_t)(sz <= avail ? sz : avail);
      break;
    }
    pos += 8 + (size_t)sz + (sz & 1);  // chunks are word aligned
  }
  DSP_REQUIRE(have_fmt && w.data_offset > 0, "no fmt/data chunk");
  DSP_REQUIRE(w.channels >= 1 && w.channels <= 128, "channels=%d outside [1, 128]", w.channels);
  DSP_REQUIRE(w.sample_rate > 0, "sample rate %d", w.sample_rate);
  if (tag == 1) {
    w.format = DSP_WAV_PCM;
    DSP_REQUIRE(w.bits == 8 || w.bits == 16 || w.bits == 24 || w.bits == 32,
                "unsupported PCM width %d", w.bits);
  } else if (tag == 3) {
    w.format = DSP_WAV_FLOAT;
    DSP_REQUIRE(w.bits == 32 || w.bits == 64, "unsupported float width %d", w.bits);
  } else if (tag == 6 || tag == 7) {  // WAVE_FORMAT_ALAW / WAVE_FORMAT_MULAW (G.711)
    w.format = tag == 6 ? DSP_WAV_ALAW : DSP_WAV_ULAW;
    DSP_REQUIRE(w.bits == 8, "G.711 samples must be 8 bits, not %d", w.bits);
  } else {
    return set_error(DSP_EINVAL, "unsupported WAVE format tag %d", tag);
  }
  w.frames = w.data_bytes / ((int64_t)w.channels * (w.bits / 8));
  *info = w;
  return DSP_OK;
}

namespace {
uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

// IEEE 754 80-bit extended (AIFF's COMM sampleRate) -> integer Hz, truncated
// as libsndfile's tenbytefloat2int does; 0 for anything not a finite rate.
int32_t ext80_to_int(const uint8_t* p) {
  const int exp = ((p[0] & 0x7F) << 8) | p[1];
  uint64_t mant = 0;
  for (int i = 0; i < 8; ++i) mant = (mant << 8) | p[2 + i];
  if ((p[0] & 0x80) || exp == 0x7FFF || mant == 0) return 0;
  const int shift = exp - 16383 - 63;  // value = mant * 2^shift
  if (shift >= 0 || shift < -63) return 0;  // >= 2^63 Hz or < 1 Hz
  const uint64_t v = mant >> (-shift);
  return v > 0x7FFFFFFFull ? 0 : (int32_t)v;
}
}  // namespace

// FORM/AIFF and FORM/AIFC (what soundfile reads through libsndfile): COMM gives
// channels, frames, width and the 80-bit rate; AIFC adds the compression
// type ('NONE'/'twos' big-endian PCM, 'sowt' little-endian PCM, 'fl32'/'fl64'
// big-endian IEEE float, 'ulaw'/'alaw' G.711); SSND holds the samples after
// its offset field.  AIFF 8-bit PCM is signed.
int aiff_parse(const uint8_t* buf, size_t len, dsp_wav_info* info) {
  DSP_REQUIRE(buf && info, "null pointer");
  DSP_REQUIRE(len >= 12 && !memcmp(buf, "FORM", 4) &&
                  (!memcmp(buf + 8, "AIFF", 4) || !memcmp(buf + 8, "AIFC", 4)),
              "not a FORM/AIFF file");
  const bool aifc = !memcmp(buf + 8, "AIFC", 4);
  bool have_comm = false;
  int64_t comm_frames = 0;
  uint8_t comp[4] = {'N', 'O', 'N', 'E'};
  dsp_wav_info w{};
  size_t pos = 12;
  while (pos + 8 <= len) {
    const uint32_t sz = be32(buf + pos + 4);
    const uint8_t* body = buf + pos + 8;
    const size_t avail = len - (pos + 8);
    if (!memcmp(buf + pos, "COMM", 4)) {
      DSP_REQUIRE(sz >= 18 && avail >= 18, "truncated COMM chunk");
      w.channels = be16(body);
      comm_frames = be32(body + 2);
      w.bits = be16(body + 6);
      w.sample_rate = ext80_to_int(body + 8);
      if (aifc) {
        DSP_REQUIRE(sz >= 22 && avail >= 22, "truncated AIFC COMM chunk");
        memcpy(comp, body + 18, 4);
      }
      have_comm = true;
    } else if (!memcmp(buf + pos, "SSND", 4)) {
      DSP_REQUIRE(have_comm, "SSND chunk before COMM chunk");
      DSP_REQUIRE(sz >= 8 && avail >= 8, "truncated SSND chunk");
      const uint32_t off = be32(body);
      const size_t chunk = sz <= avail ? sz : avail;  // a streamed size may run past the end
      DSP_REQUIRE((size_t)off + 8 <= chunk, "SSND offset %u past the chunk", off);
      w.data_offset = (int64_t)(pos + 16 + off);
      w.data_bytes = (int64_t)(chunk - 8 - off);
      break;
    }
    pos += 8 + (size_t)sz + (sz & 1);
  }
  DSP_REQUIRE(have_comm && w.data_offset > 0, "no COMM/SSND chunk");
  DSP_REQUIRE(w.channels >= 1 && w.channels <= 128, "channels=%d outside [1, 128]", w.channels);
  DSP_REQUIRE(w.sample_rate > 0, "sample rate not a positive integer");
  int width = 0;
  if (!memcmp(comp, "NONE", 4) || !memcmp(comp, "twos", 4) || !memcmp(comp, "sowt", 4)) {
    DSP_REQUIRE(w.bits == 8 || w.bits == 16 || w.bits == 24 || w.bits == 32,
                "unsupported PCM width %d", w.bits);
    const bool le = !memcmp(comp, "sowt", 4);
    w.format = DSP_WAV_PCM | (le ? 0 : DSP_AUDIO_BE) | (w.bits == 8 ? DSP_AUDIO_S8 : 0);
    width = w.bits / 8;
  } else if (!memcmp(comp, "fl32", 4) || !memcmp(comp, "FL32", 4)) {
    w.format = DSP_WAV_FLOAT | DSP_AUDIO_BE;
    w.bits = 32;
    width = 4;
  } else if (!memcmp(comp, "fl64", 4) || !memcmp(comp, "FL64", 4)) {
    w.format = DSP_WAV_FLOAT | DSP_AUDIO_BE;
    w.bits = 64;
    width = 8;
  } else if (!memcmp(comp, "ulaw", 4) || !memcmp(comp, "ULAW", 4) ||
             !memcmp(comp, "alaw", 4) || !memcmp(comp, "ALAW", 4)) {
    const bool mu = comp[0] == 'u' || comp[0] == 'U';
    w.format = (mu ? DSP_WAV_ULAW : DSP_WAV_ALAW) | DSP_AUDIO_BE;
    w.bits = 8;  // COMM says 16 (the decoded width); one byte per sample is stored
    width = 1;
  } else {
    return set_error(DSP_EINVAL, "unsupported AIFF-C compression '%c%c%c%c'", comp[0], comp[1],
                     comp[2], comp[3]);
  }
  const int64_t stored = w.data_bytes / ((int64_t)w.channels * width);
  w.frames = comm_frames < stored ? comm_frames : stored;
  *info = w;
  return DSP_OK;
}

int audio_parse(const uint8_t* buf, size_t len, dsp_wav_info* info) {
  DSP_REQUIRE(buf && info, "null pointer");
  if (len >= 4 && !memcmp(buf, "FORM", 4)) return aiff_parse(buf, len, info);
  return wav_parse(buf, len, info);
}

int wav_header_pcm16(uint8_t* out, int32_t fs, int32_t channels, int64_t frames) {
  DSP_REQUIRE(out && fs > 0 && channels >= 1 && channels <= 65535 && frames >= 0,
              "bad header arguments");
  DSP_REQUIRE(frames <= ((int64_t)UINT32_MAX - 36) / (2 * (int64_t)channels),
              "data too large for RIFF");
  DSP_REQUIRE((int64_t)fs * channels * 2 <= (int64_t)UINT32_MAX, "byte rate too large for RIFF");
  const int64_t data = frames * channels * 2;
  memcpy(out, "RIFF", 4);
  wr32(out + 4, (uint32_t)(36 + data));
  memcpy(out + 8, "WAVEfmt ", 8);
  wr32(out + 16, 16);
  wr16(out + 20, 1);
  wr16(out + 22, (uint16_t)channels);
  wr32(out + 24, (uint32_t)fs);
  wr32(out + 28, (uint32_t)((int64_t)fs * channels * 2));
  wr16(out + 32, (uint16_t)(channels * 2));
  wr16(out + 34, 16);
  memcpy(out + 36, "data", 4);
  wr32(out + 40, (uint32_t)data);
  return DSP_OK;
}

int launch_pcm_mono(const void* pcm, int format, int bits, int channels, int64_t B,
                    int64_t frames, int64_t ld_bytes, float* out, int64_t ld_out, hipStream_t s) {
  DSP_REQUIRE(B >= 0 && frames >= 0 && channels >= 1 && channels <= 128, "bad sizes");
  DSP_REQUIRE(bits == 8 || bits == 16 || bits == 24 || bits == 32 || bits == 64,
              "unsupported sample width %d", bits);
  DSP_REQUIRE(ld_bytes >= frames * channels * (bits / 8) && ld_out >= frames,
              "leading dimension too small");
  if (B == 0 || frames == 0) return DSP_OK;
  DSP_REQUIRE(pcm && out, "null pointer");
  const uint8_t* p = static_cast<const uint8_t*>(pcm);
#define DSP_PCM(F, BI, FLAGS)                                                                 \
  if (format == ((F) | (FLAGS)) && bits == BI) {                                              \
    return for_row_ranges(B, [&](int64_t b0, int64_t nb) {                                    \
      hipLaunchKernelGGL((k_pcm_mono<F, BI, ((FLAGS) & DSP_AUDIO_BE) != 0,                    \
                                     ((FLAGS) & DSP_AUDIO_S8) != 0>),                         \
                         dim3(io_blocks(frames), (unsigned)nb), dim3(kIoNT), 0, s,            \
                         p + b0 * ld_bytes, channels, frames, ld_bytes, out + b0 * ld_out,    \
                         ld_out);                                                             \
      DSP_LAUNCHED("k_pcm_mono");                                                             \
      return DSP_OK;                                                                          \
    });                                                                                       \
  }
  DSP_PCM(DSP_WAV_PCM, 8, 0)                       // WAV: unsigned 8-bit
  DSP_PCM(DSP_WAV_PCM, 8, DSP_AUDIO_S8)            // AIFF: signed 8-bit
  DSP_PCM(DSP_WAV_PCM, 8, DSP_AUDIO_S8 | DSP_AUDIO_BE)
  DSP_PCM(DSP_WAV_PCM, 16, 0)
  DSP_PCM(DSP_WAV_PCM, 24, 0)
  DSP_PCM(DSP_WAV_PCM, 32, 0)
  DSP_PCM(DSP_WAV_PCM, 16, DSP_AUDIO_BE)
  DSP_PCM(DSP_WAV_PCM, 24, DSP_AUDIO_BE)
  DSP_PCM(DSP_WAV_PCM, 32, DSP_AUDIO_BE)
  DSP_PCM(DSP_WAV_FLOAT, 32, 0)
  DSP_PCM(DSP_WAV_FLOAT, 64, 0)
  DSP_PCM(DSP_WAV_FLOAT, 32, DSP_AUDIO_BE)
  DSP_PCM(DSP_WAV_FLOAT, 64, DSP_AUDIO_BE)
  DSP_PCM(DSP_WAV_ULAW, 8, 0)
  DSP_PCM(DSP_WAV_ALAW, 8, 0)
  DSP_PCM(DSP_WAV_ULAW, 8, DSP_AUDIO_BE)           // AIFF-C 'ulaw' / 'alaw' (byte order moot)
  DSP_PCM(DSP_WAV_ALAW, 8, DSP_AUDIO_BE)
#undef DSP_PCM
  return set_error(DSP_EINVAL, "unsupported sample format 0x%x / %d bits", format, bits);
}

namespace {
// Workspace of the batched loader: the device copy of the descriptor table,
// then the block-maxima table [B][io_blocks(width)].
struct PcmBatchWs {
  size_t rows_off, max_off, total;
};
PcmBatchWs pcm_batch_ws(int64_t B, int64_t width) {
  PcmBatchWs w;
  w.rows_off = 0;
  const size_t rb = mul_sat((size_t)B, sizeof(dsp_pcm_row));
  w.max_off = rb == SIZE_MAX ? SIZE_MAX : (rb + 255) & ~(size_t)255;
  const size_t mb = mul_sat((size_t)B, (size_t)io_blocks(width), sizeof(uint32_t));
  w.total = (w.max_off == SIZE_MAX || mb == SIZE_MAX) ? SIZE_MAX : add_sat(w.max_off, mb);
  return w;
}
bool pcm_supported(int format, int bits) {
  switch (pcm_key(format, bits)) {
    case pcm_key(DSP_WAV_PCM, 8): case pcm_key(DSP_WAV_PCM | DSP_AUDIO_S8, 8):
    case pcm_key(DSP_WAV_PCM | DSP_AUDIO_S8 | DSP_AUDIO_BE, 8):
    case pcm_key(DSP_WAV_PCM, 16): case pcm_key(DSP_WAV_PCM, 24): case pcm_key(DSP_WAV_PCM, 32):
    case pcm_key(DSP_WAV_PCM | DSP_AUDIO_BE, 16): case pcm_key(DSP_WAV_PCM | DSP_AUDIO_BE, 24):
    case pcm_key(DSP_WAV_PCM | DSP_AUDIO_BE, 32):
    case pcm_key(DSP_WAV_FLOAT, 32): case pcm_key(DSP_WAV_FLOAT, 64):
    case pcm_key(DSP_WAV_FLOAT | DSP_AUDIO_BE, 32): case pcm_key(DSP_WAV_FLOAT | DSP_AUDIO_BE, 64):
    case pcm_key(DSP_WAV_ULAW, 8): case pcm_key(DSP_WAV_ALAW, 8):
    case pcm_key(DSP_WAV_ULAW | DSP_AUDIO_BE, 8): case pcm_key(DSP_WAV_ALAW | DSP_AUDIO_BE, 8):
      return true;
    default:
      return false;
  }
}
}  // namespace

size_t pcm_batch_workspace_bytes(int64_t B, int64_t width) {
  if (B <= 0 || width < 0) return 0;
  return pcm_batch_ws(B, width).total;
}

int launch_pcm_batch(const void* pcm, size_t pcm_bytes, const dsp_pcm_row* rows, int64_t B,
                     int64_t width, float* out, int64_t ld_out, double threshold,
                     uint32_t* peak_out, void* ws, size_t ws_bytes, hipStream_t s) {
  DSP_REQUIRE(B >= 0 && width >= 0 && ld_out >= width, "bad sizes");
  if (B == 0) return DSP_OK;
  DSP_REQUIRE(rows && out && peak_out && ws, "null pointer");
  for (int64_t b = 0; b < B; ++b) {
    const dsp_pcm_row& r = rows[b];
    DSP_REQUIRE(r.channels >= 1 && r.channels <= 128, "row %lld: channels=%d outside [1, 128]",
                (long long)b, r.channels);
    DSP_REQUIRE(pcm_supported(r.format, r.bits), "row %lld: unsupported sample format 0x%x / %d bits",
                (long long)b, r.format, r.bits);
    DSP_REQUIRE(r.frames >= 0 && r.frames <= width, "row %lld: %lld frames outside [0, width %lld]",
                (long long)b, (long long)r.frames, (long long)width);
    const int64_t nbytes = r.frames * r.channels * (r.bits / 8);
    DSP_REQUIRE(r.offset >= 0 && (uint64_t)r.offset <= pcm_bytes &&
                    (uint64_t)nbytes <= pcm_bytes - (uint64_t)r.offset,
                "row %lld: samples [%lld, +%lld) outside the %zu-byte buffer", (long long)b,
                (long long)r.offset, (long long)nbytes, pcm_bytes);
    DSP_REQUIRE(nbytes == 0 || pcm, "null pointer");
  }
  const PcmBatchWs w = pcm_batch_ws(B, width);
  DSP_REQUIRE(ws_bytes >= w.total, "loader workspace too small: %zu < %zu bytes", ws_bytes,
              w.total);
  DSP_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 255) == 0, "loader workspace not 256-B aligned");
  char* base = static_cast<char*>(ws);
  dsp_pcm_row* drows = reinterpret_cast<dsp_pcm_row*>(base + w.rows_off);
  uint32_t* bmax = reinterpret_cast<uint32_t*>(base + w.max_off);
  DSP_HIP(hipMemcpyAsync(drows, rows, (size_t)B * sizeof(dsp_pcm_row), hipMemcpyHostToDevice, s));
  const unsigned nbx = io_blocks(width);
  if (width == 0) {
    // nothing to decode: every peak is 0
    DSP_HIP(hipMemsetAsync(peak_out, 0, (size_t)B * sizeof(uint32_t), s));
    return DSP_OK;
  }
  const uint8_t* p = static_cast<const uint8_t*>(pcm);
  return for_row_ranges(B, [&](int64_t b0, int64_t nb) {
    {
      TraceScope trace("pcm_batch", s);
      hipLaunchKernelGGL(k_pcm_batch, dim3(nbx, (unsigned)nb), dim3(kIoNT), 0, s, p, drows, b0,
                         width, out + b0 * ld_out, ld_out, bmax);
      DSP_LAUNCHED("k_pcm_batch");
    }
    TraceScope trace("pcm_batch_scale", s);
    hipLaunchKernelGGL(k_scale_batch, dim3(nbx, (unsigned)nb), dim3(kIoNT), 0, s,
                       out + b0 * ld_out, ld_out, drows, b0, bmax, (int)nbx, threshold, peak_out);
    DSP_LAUNCHED("k_scale_batch");
    return DSP_OK;
  });
}

int launch_peak_normalize(float* x, int64_t B, int64_t n, int64_t ld, double threshold,
                          uint32_t* peak, hipStream_t s) {
  DSP_REQUIRE(B >= 0 && n >= 0 && ld >= n, "bad sizes");
  if (B == 0) return DSP_OK;
  DSP_REQUIRE(x && peak, "null pointer");
  TraceScope trace("peak_normalize", s);
  if (int rc = absmax(x, B, n, ld, peak, false, s)) return rc;
  if (n == 0) return DSP_OK;
  return for_row_ranges(B, [&](int64_t b0, int64_t nb) {
    hipLaunchKernelGGL(k_scale, dim3(io_blocks(n), (unsigned)nb), dim3(kIoNT), 0, s, x + b0 * ld,
                       n, ld, peak + b0, threshold);
    DSP_LAUNCHED("k_scale");
    return DSP_OK;
  });
}

// Host <-> device dtype edges of the drop-in (modules/dsp_core.py): numpy's
// float64 arrays narrowed to the kernels' float32 and their float32 results
// widened back, on the device (round to nearest even, as numpy's astype;
// float32 -> float64 is exact).  Flat arrays, 16-byte vectors where both
// pointers allow, grid-stride.
template <class TI, class TO>
__global__ __launch_bounds__(kIoNT) void k_convert(const TI* __restrict__ in, TO* __restrict__ out,
                                                   int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kIoNT;
  for (int64_t i = (int64_t)blockIdx.x * kIoNT + threadIdx.x; i < n; i += stride)
    out[i] = (TO)in[i];
}

template <class TI, class TO>
int launch_convert(const TI* in, TO* out, int64_t n, hipStream_t s) {
  DSP_REQUIRE(n >= 0, "bad size");
  if (n == 0) return DSP_OK;
  DSP_REQUIRE(in && out, "null pointer");
  const int64_t blocks = std::min<int64_t>(ceil_div(n, (int64_t)kIoNT), 8192);
  TraceScope trace("convert", s);
  hipLaunchKernelGGL((k_convert<TI, TO>), dim3((unsigned)blocks), dim3(kIoNT), 0, s, in, out, n);
  DSP_LAUNCHED("k_convert");
  return DSP_OK;
}

int launch_convert_f64_f32(const double* in, float* out, int64_t n, hipStream_t s) {
  return launch_convert(in, out, n, s);
}
int launch_convert_f32_f64(const float* in, double* out, int64_t n, hipStream_t s) {
  return launch_convert(in, out, n, s);
}

int launch_quantize_pcm16(const float* z, int16_t* out, int64_t B, int64_t n, int64_t ld_z,
                          int64_t ld_out, uint32_t* peak, int precision, hipStream_t s) {
  DSP_REQUIRE(B >= 0 && n >= 0 && ld_z >= n && ld_out >= n, "bad sizes");
  DSP_REQUIRE(precision == 32 || precision == 64, "precision %d is not 32 or 64", precision);
  if (B == 0) return DSP_OK;
  DSP_REQUIRE(z && out && peak, "null pointer");
  TraceScope trace("quantize16", s);
  if (int rc = absmax(z, B, n, ld_z, peak, true, s)) return rc;
  if (n == 0) return DSP_OK;
  return for_row_ranges(B, [&](int64_t b0, int64_t nb) {
    const dim3 grid(io_blocks(n), (unsigned)nb);
    if (precision == 32)
      hipLaunchKernelGGL(k_quantize16<true>, grid, dim3(kIoNT), 0, s, z + b0 * ld_z, n, ld_z,
                         out + b0 * ld_out, ld_out, peak + b0);
    else
      hipLaunchKernelGGL(k_quantize16<false>, grid, dim3(kIoNT), 0, s, z + b0 * ld_z, n, ld_z,
                         out + b0 * ld_out, ld_out, peak + b0);
    DSP_LAUNCHED("k_quantize16");
    return DSP_OK;
  });
}

}  // namespace dsp
