// Microbenchmark (gfx950): does an f32 MFMA stream run concurrently with an
// fp64 VALU FMA stream on the same SIMD?  Workgroups of 8 waves (two per SIMD:
// waves w and w+4 share one), one workgroup per CU.  Modes:
//   0: waves 0-3 MFMA, 4-7 idle      1: waves 0-3 idle, 4-7 fp64 FMA
//   2: waves 0-3 MFMA, 4-7 fp64 FMA  (concurrent: time ~ max of 0 and 1)
//   3: waves 0-3 fp64 FMA, 4-7 fp64 FMA (VALU contention reference)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_mfma_valu tools/ubench_mfma_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ float mfma_loop(int iters) {
  f32x4 acc[4] = {};
  const float a = threadIdx.x * 1e-3f, b = 0.5f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) s += acc[c].x + acc[c].y + acc[c].z + acc[c].w;
  return s;
}

__device__ float fma64_loop(int iters) {
  double x[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = fma(x[c], 0.999, 0.001);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += x[c];
  return (float)s;
}

template <int MODE>
__global__ __launch_bounds__(512) void k(float* out, int it_mfma, int it_valu) {
  const int w = threadIdx.x / 64;
  float r = 0.f;
  if (w < 4) {
    if (MODE == 0 || MODE == 2) r = mfma_loop(it_mfma);
    if (MODE == 3) r = fma64_loop(it_valu);
  } else {
    if (MODE >= 1) r = fma64_loop(it_valu);
  }
  out[blockIdx.x * 512 + threadIdx.x] = r;
}

template <int MODE>
float run(float* out, int im, int iv) {
  hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(512), 0, 0, out, 10, 10);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(512), 0, 0, out, im, iv);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 256 * 512 * sizeof(float));
  const int im = 20000, iv = 20000;
  const float t0 = run<0>(out, im, iv), t1 = run<1>(out, im, iv), t2 = run<2>(out, im, iv),
              t3 = run<3>(out, im, iv);
  // 16x16x4 f32 = 1024 MAC; 4 per iteration per wave; 1024 waves of MFMA.
  const double mfma_tf = 1024.0 * im * 4 * 1024 * 2 / (t0 * 1e-3) / 1e12;
  const double valu_tf = 1024.0 * iv * 8 * 64 * 2 / (t1 * 1e-3) / 1e12;
  printf("mode0 MFMA f32 only   %.3f ms  (%.1f TFLOP/s)\n", t0, mfma_tf);
  printf("mode1 fp64 VALU only  %.3f ms  (%.1f TFLOP/s)\n", t1, valu_tf);
  printf("mode2 both, same SIMD %.3f ms  (max %.3f, sum %.3f)\n", t2, t0 > t1 ? t0 : t1, t0 + t1);
  printf("mode3 fp64 x2 waves   %.3f ms\n", t3);
  return 0;
}
