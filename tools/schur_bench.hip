// Development microbenchmark (not part of the library): cycles per point of k_schur's consumer loop
// (schur_wave_batch, slam-robot_amd/csrc/schur_tiles.h) on one workgroup of 4 waves, synthetic C5-like batch
// (21 points, first block 0-1, spans 6-18, window 7 tiles).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Islam-robot_amd/csrc -Iinclude tools/schur_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "schur_tiles.h"
using namespace sg;
__global__ __launch_bounds__(256) void k_bench(const double* Xg, const int4* pg, int npts, int ntw, int reps,
                                               double* out, unsigned long long* cyc) {
  __shared__ double Xb[kSchurXCap + 64 * kSchurTW];
  __shared__ double wsh[4 * kSchurBatchPts];
  __shared__ int4 pinf[kSchurBatchPts];
  const int tid = threadIdx.x, lane = tid & 63, cw = tid >> 6;
  for (int i = tid; i < kSchurXCap + 64 * kSchurTW; i += 256) Xb[i] = i < kSchurXCap ? Xg[i] : 0.0;
  if (tid < 4 * kSchurBatchPts) wsh[tid] = 0.5 + tid;
  if (tid < npts) pinf[tid] = pg[tid];
  __syncthreads();
  f64x4 acc[kSchurTPW];
  for (int s = 0; s < kSchurTPW; ++s) acc[s] = f64x4{0, 0, 0, 0};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    switch (cw) {
      case 0: schur_wave_batch<0>(acc, Xb, wsh, pinf, npts, lane); break;
      case 1: schur_wave_batch<1>(acc, Xb, wsh, pinf, npts, lane); break;
      case 2: schur_wave_batch<2>(acc, Xb, wsh, pinf, npts, lane); break;
      default: schur_wave_batch<3>(acc, Xb, wsh, pinf, npts, lane); break;
    }
  }
  mfma_drain();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int k = 0; k < kSchurTPW; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[tid] = s;
  if (lane == 0) cyc[cw] = t1 - t0;
}
int main() {
  std::vector<double> X(kSchurXCap);
  for (size_t i = 0; i < X.size(); ++i) X[i] = 1e-3 * (double)((i * 2654435761u) % 1000);
  std::vector<int4> P;
  int xoff = 0, mf = 0, mr = 0;
  for (int t = 0; t < 21; ++t) {
    const int pf = t % 2, span = 6 + (t * 7) % 13;
    const int jhi = (6 * (pf + span) - 1) / 16;
    if (xoff + 64 * (jhi + 1) > kSchurXCap) break;
    P.push_back(make_int4(0, 0, xoff, jhi));
    xoff += 64 * (jhi + 1);
    mf += (jhi + 1) * (jhi + 2) / 2;
    mr += jhi + 1;
  }
  const int npts = (int)P.size(), ntw = 7, reps = 200;
  double *Xg, *out; int4* pg; unsigned long long* cyc;
  (void)hipMalloc(&Xg, X.size() * 8); (void)hipMalloc(&pg, P.size() * 16);
  (void)hipMalloc(&out, 256 * 8); (void)hipMalloc(&cyc, 64);
  (void)hipMemcpy(Xg, X.data(), X.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(pg, P.data(), P.size() * 16, hipMemcpyHostToDevice);
  printf("%d points, %d tile + %d rhs MFMAs per pass (%.1f per wave-point)\n", npts, mf, mr, (mf + mr) / 4.0 / npts);
  hipLaunchKernelGGL(k_bench, dim3(1), dim3(256), 0, 0, Xg, pg, npts, ntw, reps, out, cyc);
  hipLaunchKernelGGL(k_bench, dim3(1), dim3(256), 0, 0, Xg, pg, npts, ntw, reps, out, cyc);
  (void)hipDeviceSynchronize();
  unsigned long long c[8];
  (void)hipMemcpy(c, cyc, 64, hipMemcpyDeviceToHost);
  printf("cycles per point: wave0 %.0f  wave1 %.0f  wave2 %.0f  wave3 %.0f   (MFMA bound %.0f)\n",
         (double)c[0] / (reps * npts), (double)c[1] / (reps * npts), (double)c[2] / (reps * npts),
         (double)c[3] / (reps * npts), 64.0 * (mf + mr) / 4.0 / npts);
  return 0;
}
