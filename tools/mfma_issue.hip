// Development microbenchmark (not part of the library): f64 MFMA issue rate of one wave when each MFMA is
// followed by (0) nothing, (1) 4 independent int VALU ops, (2) a v_readlane + scalar ops + a scalar branch,
// (3) an LDS read, (4) 2 independent f64 VALU ops.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_issue.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ __launch_bounds__(64) void k_issue(double* out, unsigned long long* cyc, int iters, int flag) {
  __shared__ double lds[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = i;
  __syncthreads();
  f64x4 acc[4];
  for (int k = 0; k < 4; ++k) acc[k] = f64x4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0, x = 1.0, y = 2.0;
  int i0 = threadIdx.x, i1 = threadIdx.x * 3, sflag = flag;
  double l = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
      if (MODE == 1) { i0 += 3; i1 ^= i0; i0 += i1; i1 += 7; asm volatile("" : "+v"(i0), "+v"(i1)); }
      if (MODE == 2) {
        const int s = __builtin_amdgcn_readlane(i0, k);
        if (s + sflag + it < 0) { i1 += 1; }
        asm volatile("" : "+v"(i1));
      }
      if (MODE == 3) { l += lds[(i0 + k * 64 + it) & 1023]; }
      if (MODE == 4) { x = x * 1.0000001; y = y * 0.9999999; asm volatile("" : "+v"(x), "+v"(y)); }
    }
    asm volatile("" : "+v"(a));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3] + i0 + i1 + l + x + y;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
template <int MODE>
void run(double* out, unsigned long long* cyc) {
  const int iters = 1000;
  hipLaunchKernelGGL(k_issue<MODE>, dim3(1), dim3(64), 0, 0, out, cyc, iters, 1);
  hipLaunchKernelGGL(k_issue<MODE>, dim3(1), dim3(64), 0, 0, out, cyc, iters, 1);
  (void)hipDeviceSynchronize();
  unsigned long long c;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("mode %d: %.1f cycles per MFMA\n", MODE, (double)c / (iters * 4));
}
int main() {
  double* out; unsigned long long* cyc;
  (void)hipMalloc(&out, 1 << 16); (void)hipMalloc(&cyc, 64);
  run<0>(out, cyc); run<1>(out, cyc); run<2>(out, cyc); run<3>(out, cyc); run<4>(out, cyc);
  return 0;
}
