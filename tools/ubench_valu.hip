// Microbenchmark: VALU issue rates on gfx950 for the chain kernel's
// instruction mix -- v_fma_f64, v_fma_f32, v_pk_fma_f32 -- at 1..8 waves per
// SIMD with 8 independent chains per lane.  Prints wave-instructions per SIMD
// per cycle (cycles from s_memtime; clock-independent) and lane-FLOP/s.
// Build: hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 -o tools/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(64) void k_valu(float* out, int iters, long long* cyc) {
  const long long t0 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
  if constexpr (KIND == 0) {  // fp64 fma
    double x[8];
    for (int c = 0; c < 8; ++c) x[c] = threadIdx.x + c;
    const double a = 0.999, b = 0.001;
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int c = 0; c < 8; ++c) x[c] = fma(x[c], a, b);
    for (int c = 0; c < 8; ++c) r += (float)x[c];
  } else if constexpr (KIND == 1) {  // fp32 fma
    float x[8];
    for (int c = 0; c < 8; ++c) x[c] = threadIdx.x + c;
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int c = 0; c < 8; ++c) x[c] = fmaf(x[c], 0.999f, 0.001f);
    for (int c = 0; c < 8; ++c) r += x[c];
  } else {  // packed fp32 fma (two lanes' worth per instruction)
    f32x2 x[8];
    for (int c = 0; c < 8; ++c) x[c] = f32x2{(float)threadIdx.x, (float)c};
    const f32x2 a = {0.999f, 0.998f}, b = {0.001f, 0.002f};
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int c = 0; c < 8; ++c) x[c] = __builtin_elementwise_fma(x[c], a, b);
    for (int c = 0; c < 8; ++c) r += x[c].x + x[c].y;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char* name, int waves_per_simd, int iters) {
  const int blocks = 1024 * waves_per_simd;  // 256 CUs x 4 SIMDs
  float* out;
  long long* cyc;
  (void)hipMalloc(&out, sizeof(float) * blocks * 64);
  (void)hipMalloc(&cyc, sizeof(long long) * blocks);
  hipLaunchKernelGGL(k_valu<KIND>, dim3(blocks), dim3(64), 0, 0, out, 100, cyc);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_valu<KIND>, dim3(blocks), dim3(64), 0, 0, out, iters, cyc);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double winstr = (double)blocks * iters * 8;  // wave-instructions
  const double lane_flop = winstr * 64 * 2 * (KIND == 2 ? 2 : 1);
  // wall-clock cycles at the measured rate: instr per SIMD per ns
  printf("%-8s waves/SIMD=%d  %8.3f ms  %6.3f wave-instr/SIMD/ns  %7.1f TFLOP/s\n", name,
         waves_per_simd, ms, winstr / 1024 / (ms * 1e6), lane_flop / ms / 1e9);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  const int iters = 20000;
  for (int w : {1, 2, 4, 8}) run<0>("fma_f64", w, iters);
  for (int w : {1, 2, 4, 8}) run<1>("fma_f32", w, iters);
  for (int w : {1, 2, 4, 8}) run<2>("pk_fma", w, iters);
  return 0;
}
