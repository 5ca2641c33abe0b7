// Probe (gfx950): range checks of 16-byte raw buffer loads/stores that straddle
// num_records -- checked per dword (the in-range head is stored/loaded, the
// rest dropped / zero).  The chain kernels rely on it for rows whose length
// is not a multiple of 4.  Build: hipcc -O2 --offload-arch=gfx950 -o probe tools/probe_buffer_oob.hip
// Result on MI355X: "store y[6..13]: -1 -1 7 8 -1 -1 -1 -1", "load x[8..11]: 108 109 0 0".
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const float* x, float* y, int n) {
  // range = n floats; lane 0 loads/stores the float4 at offset n-2 (straddles the end)
  __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, n * 4, 0x00020000);
  __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(y, 0, n * 4, 0x00020000);
  if (threadIdx.x == 0) {
    f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rx, (n - 2) * 4, 0, 0);
    y[n + 4] = v.x; y[n + 5] = v.y; y[n + 6] = v.z; y[n + 7] = v.w;
    u32x4 d = {__float_as_uint(7.f), __float_as_uint(8.f), __float_as_uint(9.f), __float_as_uint(10.f)};
    __builtin_amdgcn_raw_buffer_store_b128(d, ry, (n - 2) * 4, 0, 0);
  }
}
int main() {
  const int n = 10;
  float h[32];
  for (int i = 0; i < 32; ++i) h[i] = 100 + i;
  float *dx, *dy;
  (void)hipMalloc(&dx, 32 * 4); (void)hipMalloc(&dy, 32 * 4);
  (void)hipMemcpy(dx, h, 128, hipMemcpyHostToDevice);
  for (int i = 0; i < 32; ++i) h[i] = -1;
  (void)hipMemcpy(dy, h, 128, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dx, dy, n);
  (void)hipMemcpy(h, dy, 128, hipMemcpyDeviceToHost);
  printf("store y[6..13]: "); for (int i = 6; i < 14; ++i) printf("%g ", h[i]);
  printf("\nload x[8..11] (x[10],x[11] out of range): %g %g %g %g\n", h[14], h[15], h[16], h[17]);
  return 0;
}
