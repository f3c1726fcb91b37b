// Development microbenchmark (not part of the library): f64 MFMA rate of waves 4-7 of a 512-thread workgroup
// while waves 0-3 (same SIMDs) run (0) nothing, (1) dependent f64 FMAs, (2) independent f64 FMAs, (3) int ops,
// (4) LDS reads.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_mix.hip -o mfma_mix
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(512) void k_mix(double* out, unsigned long long* cyc, int iters, int mode) {
  __shared__ double lds[4096];
  const int wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4096; i += 512) lds[i] = i;
  f64x4 acc[4];
  for (int k = 0; k < 4; ++k) acc[k] = f64x4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0;
  double x[8];
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x + k;
  int ix = threadIdx.x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (wave >= 4) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
      asm volatile("" : "+v"(a));
    }
  } else if (mode == 1) {
    for (int it = 0; it < iters * 16; ++it) x[0] = fma(x[0], 1.0000001, 1e-9);
  } else if (mode == 2) {
    for (int it = 0; it < iters * 4; ++it)
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = fma(x[k], 1.0000001, 1e-9);
  } else if (mode == 3) {
    for (int it = 0; it < iters * 32; ++it) { ix = ix * 1664525 + 1013904223; asm volatile("" : "+v"(ix)); }
  } else if (mode == 4) {
    double s = 0;
    for (int it = 0; it < iters * 8; ++it) { s += lds[(ix + it * 64) & 4095]; }
    x[0] = s;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3] + x[0] + x[7] + ix;
  if ((threadIdx.x & 63) == 0) cyc[wave] = t1 - t0;
}
int main() {
  double* out; unsigned long long* cyc;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMalloc(&cyc, 64 * 8);
  const char* names[] = {"idle", "dependent f64 fma", "independent f64 fma", "int ops", "lds reads"};
  for (int mode = 0; mode < 5; ++mode) {
    const int iters = 1000;
    hipLaunchKernelGGL(k_mix, dim3(1), dim3(512), 0, 0, out, cyc, iters, mode);
    hipLaunchKernelGGL(k_mix, dim3(1), dim3(512), 0, 0, out, cyc, iters, mode);
    (void)hipDeviceSynchronize();
    unsigned long long c[8];
    (void)hipMemcpy(c, cyc, 64, hipMemcpyDeviceToHost);
    printf("%-22s MFMA wave: %.1f cycles/MFMA   other wave: %llu cycles total\n", names[mode],
           (double)c[4] / (iters * 4), c[0]);
  }
  return 0;
}
