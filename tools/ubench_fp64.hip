// Microbenchmark: fp64 / fp32 FMA throughput and dependent latency on gfx950.
// Build: hipcc -O3 --offload-arch=gfx950 -o ubench_fp64 ubench_fp64.hip
// Each lane runs CH independent FMA chains of ITERS steps; reports wave-instr/clk.
#include <hip/hip_runtime.h>

#include <cstdio>

template <typename T, int CH>
__global__ __launch_bounds__(256) void k_chain(T* out, int iters, T a, T b) {
  T x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = (T)(threadIdx.x + c);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = x[c] * a + b;  // fma
  }
  T s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename T, int CH>
void run(const char* name, int blocks, int iters) {
  T* out;
  hipMalloc(&out, sizeof(T) * blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_chain<T, CH><<<blocks, 256>>>(out, 10, (T)0.999, (T)0.001);
  hipEventRecord(e0);
  k_chain<T, CH><<<blocks, 256>>>(out, iters, (T)0.999, (T)0.001);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double lane_ops = (double)blocks * 256 * iters * CH;
  double waves_per_simd = blocks * 4.0 / 1024.0;
  printf("%-6s CH=%2d blocks=%6d waves/SIMD=%5.2f  %8.3f ms  %8.2f T lane-FMA/s (%.1f TFLOPS)\n",
         name, CH, blocks, waves_per_simd, ms, lane_ops / ms / 1e9, 2 * lane_ops / ms / 1e9);
  hipFree(out);
}

int main() {
  const int iters = 20000;
  for (int blocks : {256, 512, 1024, 2048, 4096}) {
    run<double, 1>("fp64", blocks, iters);
    run<double, 2>("fp64", blocks, iters);
    run<double, 4>("fp64", blocks, iters);
    run<double, 8>("fp64", blocks, iters);
  }
  for (int blocks : {256, 1024, 4096}) {
    run<float, 1>("fp32", blocks, iters);
    run<float, 4>("fp32", blocks, iters);
    run<float, 8>("fp32", blocks, iters);
  }
  return 0;
}
