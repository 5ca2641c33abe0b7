// Microbenchmark (gfx950): which matrix-core streams run concurrently with
// which VALU streams on the same SIMD?  Workgroups of 8 waves (waves w and
// w+4 share a SIMD), one workgroup per CU.  Each line times stream A on waves
// 0-3 and stream B on waves 4-7 (either may be idle); "max" / "sum" are the
// two streams' solo times: concurrent execution shows up as ~max.
//   MFMA f32  v_mfma_f32_16x16x4_f32      MFMA f16  v_mfma_f32_16x16x32_f16
//   fp64      v_fma_f64 (8 chains)        pk32      v_pk_fma_f32 (8 chains)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_mfma_mix tools/ubench_mfma_mix.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

enum { IDLE = 0, MF32 = 1, MF16 = 2, F64 = 3, PK32 = 4 };

__device__ float s_mf32(int iters) {
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

__device__ float s_mf16(int iters) {
  f32x4 acc[4] = {};
  f16x8 a, b;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = (_Float16)(threadIdx.x * 1e-3f + k);
    b[k] = (_Float16)0.5f;
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) s += acc[c].x + acc[c].y + acc[c].z + acc[c].w;
  return s;
}

__device__ float s_f64(int iters) {
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

__device__ float s_pk32(int iters) {
  f32x2 x[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = f32x2{(float)threadIdx.x + c, (float)c};
  const f32x2 m = f32x2{0.999f, 0.998f}, d = f32x2{0.001f, 0.002f};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = __builtin_elementwise_fma(x[c], m, d);
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += x[c].x + x[c].y;
  return s;
}

__device__ float stream(int kind, int iters) {
  switch (kind) {
    case MF32: return s_mf32(iters);
    case MF16: return s_mf16(iters);
    case F64: return s_f64(iters);
    case PK32: return s_pk32(iters);
    default: return 0.f;
  }
}

__global__ __launch_bounds__(512) void k(float* out, int ka, int ia, int kb, int ib) {
  const int w = threadIdx.x / 64;
  const float r = w < 4 ? stream(ka, ia) : stream(kb, ib);
  out[blockIdx.x * 512 + threadIdx.x] = r;
}

float run(float* out, int ka, int ia, int kb, int ib) {
  hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, out, ka, 10, kb, 10);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, out, ka, ia, kb, ib);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 256 * 512 * sizeof(float));
  const char* names[] = {"idle", "MFMA f32", "MFMA f16", "fp64 FMA", "pk_fma f32"};
  // iteration counts sized for a few ms each
  const int it[] = {0, 20000, 20000, 20000, 20000};
  float solo[5] = {0};
  for (int s = 1; s <= 4; ++s) {
    solo[s] = run(out, s, it[s], IDLE, 0);
    printf("%-12s solo      %.3f ms\n", names[s], solo[s]);
  }
  const int pairs[][2] = {{MF32, F64}, {MF16, F64}, {MF32, PK32}, {MF16, PK32},
                          {F64, F64},  {PK32, PK32}, {F64, PK32}};
  for (auto& p : pairs) {
    const float t = run(out, p[0], it[p[0]], p[1], it[p[1]]);
    const float mx = solo[p[0]] > solo[p[1]] ? solo[p[0]] : solo[p[1]];
    printf("%-12s + %-12s %.3f ms  (max %.3f, sum %.3f)\n", names[p[0]], names[p[1]], t, mx,
           solo[p[0]] + solo[p[1]]);
  }
  return 0;
}
