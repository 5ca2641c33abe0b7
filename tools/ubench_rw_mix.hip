// HBM ceiling by read:write mix (gfx950): streaming float4 kernels that read
// R and write W bytes per element, nt cache policy like the chain kernel, over
// multi-GB buffers.  The chain kernel's mix is 1 read : 2 writes (x in; y, z
// out), which a 1:1 copy ceiling does not describe.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_rw_mix tools/ubench_rw_mix.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Each thread handles float4 i of every stream: NR read streams, NW write streams.
template <int NR, int NW>
__global__ __launch_bounds__(256) void k(const f32x4* __restrict__ in, f32x4* __restrict__ out,
                                         long n4, float s) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 v = {s, s, s, s};
#pragma unroll
    for (int r = 0; r < NR; ++r) v += __builtin_nontemporal_load(in + r * n4 + i);
#pragma unroll
    for (int w = 0; w < NW; ++w) __builtin_nontemporal_store(v * (float)(w + 1), out + w * n4 + i);
    if (NW == 0 && v.x == 12345.f) out[i] = v;  // keeps the read-only loads alive
  }
}

static bool g_json = false;

template <int NR, int NW>
double run(const f32x4* in, f32x4* out, long n4, int grid) {
  hipLaunchKernelGGL((k<NR, NW>), dim3(grid), dim3(256), 0, 0, in, out, n4, 1.f);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int reps = 20;
  (void)hipEventRecord(e0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k<NR, NW>), dim3(grid), dim3(256), 0, 0, in, out, n4, 1.f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)(NR + NW) * n4 * 16;
  const double gbs = bytes / (ms / reps * 1e-3) / 1e9;
  if (!g_json) printf("read:write %d:%d  grid %6d  %.3f ms  %.0f GB/s\n", NR, NW, grid, ms / reps, gbs);
  return gbs;
}

// --json: one line {"r1w2_gbs": best 1:2 rate over the grids, "r1w1_gbs": ...}
// (bench.py's ceiling for the chain kernel's mix).
int main(int argc, char** argv) {
  // --burn S: the 1 : 2 stream back to back for S seconds (power / clock
  // readings under a pure HBM load, tools/gpu_power_stream.sh)
  const bool burn = argc > 2 && argv[1][2] == 'b';
  g_json = argc > 1 && argv[1][0] == '-';
  const long n4 = (1L << 30) / 16;  // 1 GiB per stream
  f32x4 *in, *out;
  if (hipMalloc(&in, 2 * n4 * 16) != hipSuccess || hipMalloc(&out, 2 * n4 * 16) != hipSuccess) return 1;
  (void)hipMemset(in, 0, 2 * n4 * 16);
  if (burn) {
    const double secs = atof(argv[2]);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    long launches = 0;
    for (float ms = 0.f; ms < secs * 1e3f;) {
      for (int r = 0; r < 200; ++r, ++launches)
        hipLaunchKernelGGL((k<1, 2>), dim3(65536), dim3(256), 0, 0, in, out, n4, 1.f);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("burn %.1f s %.0f GB/s\n", ms / 1e3, 3.0 * n4 * 16 * launches / (ms * 1e-3) / 1e9);
      fflush(stdout);
    }
    return 0;
  }
  double b12 = 0, b11 = 0;
  for (int grid : {4096, 16384, 65536}) {
    if (!g_json) run<1, 0>(in, out, n4, grid);
    b11 = std::max(b11, run<1, 1>(in, out, n4, grid));
    b12 = std::max(b12, run<1, 2>(in, out, n4, grid));
    if (!g_json) {
      run<0, 1>(in, out, n4, grid);
      run<2, 1>(in, out, n4, grid);
    }
  }
  if (g_json) printf("{\"r1w2_gbs\": %.1f, \"r1w1_gbs\": %.1f}\n", b12, b11);
  (void)hipFree(in);
  (void)hipFree(out);
  return 0;
}
