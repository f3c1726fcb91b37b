// Development microbenchmark (not part of the library): issue rate of v_mfma_f64_16x16x4f64 on gfx950 with
// K independent accumulators per wave, for 1..4 waves per SIMD (workgroup of 64 * 4 * wps threads on one CU).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o tools/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int K>
__global__ void k_rate(double* out, unsigned long long* cyc, int iters) {
  f64x4 acc[K];
  for (int k = 0; k < K; ++k) acc[k] = f64x4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    asm volatile("" : "+v"(a));
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int k = 0; k < K; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int K>
void run(double* out, unsigned long long* cyc, int wps) {
  const int iters = 2000;
  hipLaunchKernelGGL(k_rate<K>, dim3(1), dim3(256 * wps), 0, 0, out, cyc, iters);
  hipLaunchKernelGGL(k_rate<K>, dim3(1), dim3(256 * wps), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const double per = (double)c / (iters * K * wps);   // cycles per MFMA per SIMD
  printf("K=%d waves/SIMD=%d: %.1f cycles per MFMA per SIMD (%.1f per wave-MFMA)\n", K, wps, per, per * wps);
}
int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&cyc, 64);
  for (int wps = 1; wps <= 4; wps *= 2) {
    run<1>(out, cyc, wps);
    run<4>(out, cyc, wps);
    run<8>(out, cyc, wps);
  }
  return 0;
}
