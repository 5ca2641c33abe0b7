// Probe: HBM rate of the four-step FFT's access shapes with no arithmetic.
// A 2^28-element float2 matrix of R rows x C columns (row pitch C); each
// workgroup copies a block of KC consecutive columns x all R rows, the thread
// mapping of k_fft4_a (c = i % KC, r = i / KC), through LDS like the FFT.
//   hipcc -O3 --offload-arch=gfx950 tools/stride_probe.hip -o tools/_stride_probe
//   ./tools/_stride_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

template <int KC, int NT, int R>
__global__ __launch_bounds__(NT) void k_copy_cols(const float2* __restrict__ src, float2* dst,
                                                  long C, int xcd) {
  extern __shared__ float2 lds[];
  long gx = blockIdx.x;
  if (xcd && (gridDim.x & 7) == 0) gx = (gx & 7) * (gridDim.x >> 3) + (gx >> 3);
  const long c0 = gx * KC;
  src += (long)blockIdx.y * R * C;
  dst += (long)blockIdx.y * R * C;
  constexpr int PER = KC * R / NT;
  float2 v[PER];
#pragma unroll
  for (int it = 0; it < PER; ++it) {  // every load in flight before the first use
    const int i = threadIdx.x + it * NT;
    v[it] = src[(long)(i / KC) * C + c0 + i % KC];
  }
#pragma unroll
  for (int it = 0; it < PER; ++it) lds[threadIdx.x + it * NT] = v[it];
  __syncthreads();
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const int i = threadIdx.x + it * NT;
    float2 w = lds[i];
    w.x += 1.f;
    dst[(long)(i / KC) * C + c0 + i % KC] = w;
  }
}

template <int KC, int NT, int R>
void run(const char* what, const float2* s, float2* d, long C, int xcd) {
  const long n = 1L << 28;
  const dim3 grid((unsigned)(C / KC), (unsigned)(n / C / R));
  const size_t shm = (size_t)KC * R * sizeof(float2);
  CK(hipFuncSetAttribute((const void*)k_copy_cols<KC, NT, R>,
                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_copy_cols<KC, NT, R>), grid, dim3(NT), shm, 0, s, d, C, xcd);
  CK(hipEventRecord(e0));
  const int reps = 5;
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((k_copy_cols<KC, NT, R>), grid, dim3(NT), shm, 0, s, d, C, xcd);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = 2.0 * n * sizeof(float2);
  std::printf("%-30s R=%5d C=%8ld KC=%2d xcd=%d  %.3f ms  %.0f GB/s\n", what, R, C, KC, xcd, ms,
              bytes / (ms * 1e-3) / 1e9);
}

int main() {
  const long n = 1L << 28;
  float2 *s, *d;
  CK(hipMalloc(&s, n * sizeof(float2)));
  CK(hipMalloc(&d, n * sizeof(float2)));
  CK(hipMemset(s, 0, n * sizeof(float2)));
  // step A of 2^28 = 2^9 x 2^19: columns of 512 rows, 4 MB apart
  run<8, 256, 512>("cols of 512, 4 MB pitch", s, d, n / 512, 1);
  run<8, 256, 512>("cols of 512, 4 MB pitch", s, d, n / 512, 0);
  run<16, 256, 512>("cols of 512, 4 MB pitch", s, d, n / 512, 1);
  // columns of 1024 rows (2^30's step A shape at 2^28 size)
  run<8, 512, 1024>("cols of 1024, 2 MB pitch", s, d, n / 1024, 1);
  // step A' shape: 512 rows 8 KB apart (C = 1024), blocks tile the matrix
  run<8, 256, 512>("cols of 512, 8 KB pitch", s, d, 1024, 1);
  // contiguous: pitch = KC, so a block is 64 KB in one piece
  run<16, 256, 512>("contiguous 64 KB blocks", s, d, 16, 0);
  CK(hipFree(s));
  CK(hipFree(d));
  return 0;
}
