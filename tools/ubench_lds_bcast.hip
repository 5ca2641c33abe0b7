// LDS read throughput of ds_read_b128 by address pattern (gfx950), to decide
// whether lanes sharing a tap row (broadcast) read it cheaper than lanes
// reading distinct rows.  One workgroup per CU-slot, 4 waves, 4096 reads per
// lane; prints ns per wave-instruction per CU.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_lds_bcast.hip -o /tmp/ub && /tmp/ub
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

// mode 0: every lane its own 16-B row (64 distinct, conflict-free)
// mode 1: all lanes the same row
// mode 2: 5 distinct rows (lane % 5), spread over banks
// mode 3: 5 distinct rows in contiguous lane groups (lane * 5 / 64)
// mode 4: 16 distinct rows (lane % 16)
template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  __shared__ f4 lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = f4{1.f * i, 2.f, 3.f, 4.f};
  __syncthreads();
  const int lane = threadIdx.x & 63;
  int row = MODE == 0 ? lane : MODE == 1 ? 0 : MODE == 2 ? (lane % 5) * 97 : MODE == 3 ? (lane * 5 / 64) * 97 : (lane % 16) * 97;
  row &= 4095;
  f4 acc = f4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      // `it` in the address keeps the loads inside the loop (no LICM)
      const f4 v = lds[(row + u * 64 * (MODE == 0 ? 1 : 0) + u * 7 + it * 11) & 4095];
      acc += v;
    }
  }
  if (acc.x == 12345.f) out[threadIdx.x] = acc.y;
}

template <int MODE>
float run(int cus) {
  float* d;
  hipMalloc(&d, 4096);
  const int iters = 256;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k<MODE>, dim3(cus * 4), dim3(256), 0, 0, d, iters);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<MODE>, dim3(cus * 4), dim3(256), 0, 0, d, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  hipFree(d);
  // wave-instructions per CU: 4 blocks x 4 waves x iters x 16
  const double per_cu = 4.0 * 4 * iters * 16;
  return (float)(ms * 1e6 / per_cu);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", cus);
  printf("mode 0 (64 distinct rows)        %.3f ns per ds_read_b128 wave-instr per CU\n", run<0>(cus));
  printf("mode 1 (one row, broadcast)      %.3f\n", run<1>(cus));
  printf("mode 2 (5 rows, lane %% 5)        %.3f\n", run<2>(cus));
  printf("mode 3 (5 rows, lane groups)     %.3f\n", run<3>(cus));
  printf("mode 4 (16 rows, lane %% 16)      %.3f\n", run<4>(cus));
  return 0;
}
