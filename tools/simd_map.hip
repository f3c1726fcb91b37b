// Development microbenchmark (not part of the library): which SIMD each wave of a 512-thread workgroup lands
// on (HW_ID.SIMD_ID), and the f64 MFMA rate when only waves 4-7 issue MFMAs.
// Build: hipcc --offload-arch=gfx950 -O3 tools/simd_map.hip -o simd_map
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(512) void k_map(int* simd, double* out, unsigned long long* cyc, int iters, int mode) {
  const int wave = threadIdx.x >> 6;
  const int hw = __builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);   // HW_ID[5:4] = SIMD_ID
  if ((threadIdx.x & 63) == 0) simd[blockIdx.x * 8 + wave] = hw;
  f64x4 acc[4];
  for (int k = 0; k < 4; ++k) acc[k] = f64x4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const bool act = mode == 0 ? wave >= 4 : (mode == 1 ? (wave & 1) : true);
  if (act)
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
      asm volatile("" : "+v"(a));
    }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 512 + threadIdx.x] = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  int* simd; double* out; unsigned long long* cyc;
  (void)hipMalloc(&simd, 8 * 4 * 1024);
  (void)hipMalloc(&out, 8 << 20);
  (void)hipMalloc(&cyc, 8 * 1024);
  for (int mode = 0; mode < 3; ++mode) {
    const int iters = 1000;
    hipLaunchKernelGGL(k_map, dim3(1), dim3(512), 0, 0, simd, out, cyc, iters, mode);
    (void)hipDeviceSynchronize();
    int h[8]; unsigned long long c;
    (void)hipMemcpy(h, simd, 32, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const int nact = mode == 2 ? 8 : 4;
    printf("mode %d simd of waves 0-7:", mode);
    for (int w = 0; w < 8; ++w) printf(" %d", (h[w] >> 4) & 3);
    printf("   %.1f cycles per MFMA-step of one wave (%d waves active, 4 MFMAs each)\n", (double)c / (iters * 4), nact);
  }
  return 0;
}
