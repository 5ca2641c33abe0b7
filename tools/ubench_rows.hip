// Microbenchmark: HBM read+write rate of the IIR's access shape on gfx950.
// One wave per channel row of n floats cut into 64 chunks of T (lane c owns
// chunk c, as k_iir_wave); per step every chunk advances TW floats and the wave
// moves the 64 x TW tile with 16-byte loads/stores, next tile's loads in flight.
// Compared with a plain contiguous grid-stride float4 copy of the same bytes.
// Build: hipcc -O3 --offload-arch=gfx950 -o ubench_rows ubench_rows.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int TW>
__global__ __launch_bounds__(64) void k_rows(const float* __restrict__ x, float* __restrict__ y,
                                             long n, long T) {
  constexpr int LPR = TW / 4;          // lanes per row
  constexpr int RPI = 64 / LPR;        // rows per instruction
  constexpr int NI = 64 / RPI;         // instructions per tile
  const long base = (long)blockIdx.x * n;
  const int lane = threadIdx.x;
  const int r0 = lane / LPR, c4 = (lane % LPR) * 4;
  float4 v[NI], w[NI];
  auto ld = [&](float4 (&d)[NI], long t0) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const long row = r0 + i * RPI;
      const long off = row * T + t0 + c4;
      d[i] = off + 3 < n && t0 < T ? *reinterpret_cast<const float4*>(x + base + off)
                                   : make_float4(0, 0, 0, 0);
    }
  };
  ld(v, 0);
  for (long t0 = 0; t0 < T; t0 += TW) {
#pragma unroll
    for (int i = 0; i < NI; ++i) w[i] = v[i];
    ld(v, t0 + TW);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const long row = r0 + i * RPI;
      const long off = row * T + t0 + c4;
      if (off + 3 < n) *reinterpret_cast<float4*>(y + base + off) = w[i];
    }
  }
}

__global__ void k_copy(const float4* __restrict__ x, float4* __restrict__ y, long n4) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    y[i] = x[i];
}

int main() {
  const long B = 4096, n = 72000, T = 1152;
  float *x, *y;
  hipMalloc(&x, B * n * 4);
  hipMalloc(&y, B * n * 4);
  hipMemset(x, 0, B * n * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-28s %8.4f ms  %6.2f TB/s (read+write)\n", name, ms, 2.0 * B * n * 4 / ms / 1e9);
  };
  timeit("contiguous copy 1024x256", [&] { k_copy<<<1024, 256>>>((const float4*)x, (float4*)y, B * n / 4); });
  timeit("contiguous copy 8192x256", [&] { k_copy<<<8192, 256>>>((const float4*)x, (float4*)y, B * n / 4); });
  timeit("rows TW=32 (IIR shape)", [&] { k_rows<32><<<B, 64>>>(x, y, n, T); });
  timeit("rows TW=64", [&] { k_rows<64><<<B, 64>>>(x, y, n, T); });
  timeit("rows TW=128", [&] { k_rows<128><<<B, 64>>>(x, y, n, T); });
  return 0;
}
