// Microbenchmark: v_mfma_f64_16x16x4_f64 throughput on gfx950 (matrix pipe),
// alone and beside an fp64 VALU FMA stream in the same wave.
// Build: hipcc -O3 --offload-arch=gfx950 -o ubench_mfma64 ubench_mfma64.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int ACC, int VALU>
__global__ __launch_bounds__(256) void k_mfma(double* out, int iters, double a, double b) {
  d4 acc[ACC > 0 ? ACC : 1];
#pragma unroll
  for (int c = 0; c < ACC; ++c) acc[c] = d4{0, 0, 0, 0};
  double x = threadIdx.x * 1e-3, y = threadIdx.x * 2e-3;
  double v[VALU > 0 ? VALU : 1];
#pragma unroll
  for (int c = 0; c < (VALU > 0 ? VALU : 1); ++c) v[c] = threadIdx.x + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < ACC; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[c], 0, 0, 0);
#pragma unroll
    for (int c = 0; c < VALU; ++c) v[c] = v[c] * a + b;
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < ACC; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
#pragma unroll
  for (int c = 0; c < VALU; ++c) s += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ACC, int VALU>
void run(int blocks, int iters) {
  double* out;
  hipMalloc(&out, sizeof(double) * blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_mfma<ACC, VALU><<<blocks, 256>>>(out, 10, 0.999, 0.001);
  hipEventRecord(e0);
  k_mfma<ACC, VALU><<<blocks, 256>>>(out, iters, 0.999, 0.001);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double waves = blocks * 4.0;
  const double mfma = waves * iters * ACC;            // wave-level MFMAs
  const double simd_cycles_per = ms * 1e-3 * 2.4e9 * 1024 / mfma;
  printf("ACC=%d VALU=%d blocks=%5d  %8.3f ms  %.2f TFLOPS mfma  %.1f SIMD-cycles/MFMA (@2.4GHz)"
         "  valu %.2f T lane-FMA/s\n",
         ACC, VALU, blocks, ms, mfma * 2048 / ms / 1e9, simd_cycles_per,
         waves * 64.0 * iters * VALU / ms / 1e9);
  hipFree(out);
}

int main() {
  const int iters = 20000;
  for (int blocks : {256, 1024}) {
    run<1, 0>(blocks, iters);
    run<4, 0>(blocks, iters);
    run<4, 8>(blocks, iters);
    run<4, 16>(blocks, iters);
    run<0, 8>(blocks, iters);
  }
  return 0;
}
