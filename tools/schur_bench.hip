// Development microbenchmark (not part of the library): cycles per point of k_schur's consumer loop
// (schur_wave_batch, slam-robot_amd/csrc/schur_tiles.h) on one workgroup of 4 waves, synthetic C5-like batch
// (21 points, first block 0-1, spans 6-18, window 7 tiles).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Islam-robot_amd/csrc -Iinclude tools/schur_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "schur_tiles.h"
using namespace sg;
// Variants of the consumer loop (argv[1]): 0 the library's schur_wave_batch; 1 three operand buffers (point
// t + 2's reads before point t's MFMAs); 2 no operand reads in the loop (point 0's operands for every point:
// the MFMA issue and slot branches alone); 3 as 2 with every point over the whole window (kSchurTPW MFMAs per
// wave and point: the cost per MFMA of the slot chain without its early exit).
template <int W>
__device__ __forceinline__ void wave_batch3(f64x4 (&acc)[kSchurTPW], const double* Xb, const double* wsh,
                                            const int4* pinf, int npts, int lane) {
  constexpr unsigned kNeed = schur_need(W);
  const int4 pv = pinf[min(lane, npts - 1)];
  double XA[kSchurTW], XB[kSchurTW], XC[kSchurTW];
#pragma unroll
  for (int j = 0; j < kSchurTW; ++j) XA[j] = XB[j] = XC[j] = 0.0;
  double wa, wb, wc;
  int ha, hb, hc;
  schur_fetch<kNeed>(Xb, wsh, pv, 0, npts, lane, XA, wa, ha);
  schur_fetch<kNeed>(Xb, wsh, pv, 1, npts, lane, XB, wb, hb);
  for (int t = 0; t < npts; t += 3) {
    schur_fetch<kNeed>(Xb, wsh, pv, t + 2, npts, lane, XC, wc, hc);
    schur_mfma<W>(acc, XA, wa, ha);
    schur_fetch<kNeed>(Xb, wsh, pv, t + 3, npts, lane, XA, wa, ha);
    schur_mfma<W>(acc, XB, wb, hb);
    schur_fetch<kNeed>(Xb, wsh, pv, t + 4, npts, lane, XB, wb, hb);
    schur_mfma<W>(acc, XC, wc, hc);
  }
}
template <int W>
__device__ __forceinline__ void wave_batch_nofetch(f64x4 (&acc)[kSchurTPW], const double* Xb, const double* wsh,
                                                   const int4* pinf, int npts, int lane, bool full) {
  constexpr unsigned kNeed = schur_need(W);
  const int4 pv = pinf[min(lane, npts - 1)];
  double XA[kSchurTW];
#pragma unroll
  for (int j = 0; j < kSchurTW; ++j) XA[j] = 0.0;
  double wa;
  int ha;
  schur_fetch<kNeed>(Xb, wsh, pv, 0, npts, lane, XA, wa, ha);
  for (int t = 0; t < npts; ++t) {
    const int h = full ? kSchurTW - 1 : __builtin_amdgcn_readlane(pv.w, t);
    schur_mfma<W>(acc, XA, wa, h);
  }
}
// mode 4: every slot of the window per point with no branches between the MFMAs (straight-line chain)
template <int W, int S>
__device__ __forceinline__ void slots_straight(f64x4 (&acc)[kSchurTPW], const double (&X)[kSchurTW], double wop) {
  if constexpr (S < kSchurTPW && W + kSchurCWaves * S < kSchurAug) {
    constexpr int u = W + kSchurCWaves * S;
    constexpr int c = schur_aug_c(u), r = schur_aug_r(u);
    if constexpr (r <= c) mfma_acc(acc[S], X[r], X[c]);
    else mfma_acc(acc[S], X[c], wop);
    slots_straight<W, S + 1>(acc, X, wop);
  }
}
template <int W>
__device__ __forceinline__ void wave_batch_straight(f64x4 (&acc)[kSchurTPW], const double* Xb, const double* wsh,
                                                    const int4* pinf, int npts, int lane) {
  constexpr unsigned kNeed = schur_need(W);
  const int4 pv = pinf[min(lane, npts - 1)];
  double XA[kSchurTW];
#pragma unroll
  for (int j = 0; j < kSchurTW; ++j) XA[j] = 0.0;
  double wa;
  int ha;
  schur_fetch<kNeed>(Xb, wsh, pv, 0, npts, lane, XA, wa, ha);
  for (int t = 0; t < npts; ++t) slots_straight<W, 0>(acc, XA, wa);
}
// mode 5: one dispatch per point (a switch on the wave's slot count) into a straight-line chain of that length
template <int W, int S, int N>
__device__ __forceinline__ void chain_n(f64x4 (&acc)[kSchurTPW], const double (&X)[kSchurTW], double wop) {
  if constexpr (S < N && S < kSchurTPW && W + kSchurCWaves * S < kSchurAug) {
    constexpr int u = W + kSchurCWaves * S;
    constexpr int c = schur_aug_c(u), r = schur_aug_r(u);
    if constexpr (r <= c) mfma_acc(acc[S], X[r], X[c]);
    else mfma_acc(acc[S], X[c], wop);
    chain_n<W, S + 1, N>(acc, X, wop);
  }
}
template <int W, int N>
__device__ __forceinline__ void chain_switch(f64x4 (&acc)[kSchurTPW], const double (&X)[kSchurTW], double wop, int ns) {
  if constexpr (N <= kSchurTPW) {
    if (ns == N) { chain_n<W, 0, N>(acc, X, wop); return; }
    chain_switch<W, N + 1>(acc, X, wop, ns);
  }
}
template <int W>
__device__ __forceinline__ void wave_batch_dispatch(f64x4 (&acc)[kSchurTPW], const double* Xb, const double* wsh,
                                                    const int4* pinf, int npts, int lane) {
  constexpr unsigned kNeed = schur_need(W);
  const int4 pv = pinf[min(lane, npts - 1)];
  double XA[kSchurTW], XB[kSchurTW];
#pragma unroll
  for (int j = 0; j < kSchurTW; ++j) XA[j] = XB[j] = 0.0;
  double wa, wb;
  int ha, hb;
  auto nsl = [](int jhi) { return (schur_aug_base(jhi + 1) - W + kSchurCWaves - 1) / kSchurCWaves; };
  schur_fetch<kNeed>(Xb, wsh, pv, 0, npts, lane, XA, wa, ha);
  for (int t = 0; t < npts; t += 2) {
    schur_fetch<kNeed>(Xb, wsh, pv, t + 1, npts, lane, XB, wb, hb);
    chain_switch<W, 1>(acc, XA, wa, nsl(ha));
    schur_fetch<kNeed>(Xb, wsh, pv, t + 2, npts, lane, XA, wa, ha);
    chain_switch<W, 1>(acc, XB, wb, nsl(hb));
  }
}
// mode 6 / 7: one dispatch per BATCH (the wave's largest slot count over the batch's points) into a loop whose
// body is a straight-line chain of that length for every point; the slots past a point's own prefix multiply
// operand columns zeroed at the fetch (mode 6; mode 7 leaves them unmasked: timing only).  With points ordered by
// (first block, last block) a batch's points share their last tile, so little is padded.
template <bool kMask, unsigned kNeed>
__device__ __forceinline__ void fetch_masked(const double* Xb, const double* wsh, const int4& pv, int t, int npts,
                                             int lane, double (&X)[kSchurTW], double& wop) {
  const int tt = min(t, npts - 1);
  const int jhi = t < npts ? __builtin_amdgcn_readlane(pv.w, tt) : -1;
  const double* xp = Xb + __builtin_amdgcn_readlane(pv.z, tt) + lane;
#pragma unroll
  for (int j = 0; j < kSchurTW; ++j)
    if ((kNeed >> j) & 1u) {
      const double v = xp[64 * j];
      X[j] = (!kMask || j <= jhi) ? v : 0.0;
    }
  const double wv = wsh[4 * tt + (lane >> 4)];
  wop = ((lane & 15) == 0 && t < npts) ? wv : 0.0;
}
template <int W, int N, bool kMask>
__device__ __forceinline__ void batch_chain(f64x4 (&acc)[kSchurTPW], const double* Xb, const double* wsh,
                                            const int4& pv, int npts, int lane) {
  constexpr unsigned kNeed = schur_need(W);
  double XA[kSchurTW], XB[kSchurTW];
#pragma unroll
  for (int j = 0; j < kSchurTW; ++j) XA[j] = XB[j] = 0.0;
  double wa, wb;
  fetch_masked<kMask, kNeed>(Xb, wsh, pv, 0, npts, lane, XA, wa);
  for (int t = 0; t < npts; t += 2) {
    fetch_masked<kMask, kNeed>(Xb, wsh, pv, t + 1, npts, lane, XB, wb);
    chain_n<W, 0, N>(acc, XA, wa);
    fetch_masked<kMask, kNeed>(Xb, wsh, pv, t + 2, npts, lane, XA, wa);
    chain_n<W, 0, N>(acc, XB, wb);
  }
}
template <int W, int N, bool kMask>
__device__ __forceinline__ void batch_switch(f64x4 (&acc)[kSchurTPW], const double* Xb, const double* wsh,
                                             const int4& pv, int npts, int lane, int ns) {
  if constexpr (N <= kSchurTPW) {
    if (ns == N) { batch_chain<W, N, kMask>(acc, Xb, wsh, pv, npts, lane); return; }
    batch_switch<W, N + 1, kMask>(acc, Xb, wsh, pv, npts, lane, ns);
  }
}
template <int W, bool kMask>
__device__ __forceinline__ void wave_batch_runs(f64x4 (&acc)[kSchurTPW], const double* Xb, const double* wsh,
                                                const int4* pinf, int npts, int lane) {
  const int4 pv = pinf[min(lane, npts - 1)];
  const int jmax = __builtin_amdgcn_readfirstlane(
      __reduce_max_sync(~0ull, lane < npts ? pv.w : 0));
  const int ns = (schur_aug_base(jmax + 1) - W + kSchurCWaves - 1) / kSchurCWaves;
  batch_switch<W, 1, kMask>(acc, Xb, wsh, pv, npts, lane, ns);
}
template <int W>
__device__ __forceinline__ void run_variant(int mode, f64x4 (&acc)[kSchurTPW], const double* Xb, const double* wsh,
                                            const int4* pinf, int npts, int lane) {
  if (mode == 1) wave_batch3<W>(acc, Xb, wsh, pinf, npts, lane);
  else if (mode == 6) wave_batch_runs<W, true>(acc, Xb, wsh, pinf, npts, lane);
  else if (mode == 7) wave_batch_runs<W, false>(acc, Xb, wsh, pinf, npts, lane);
  else if (mode == 5) wave_batch_dispatch<W>(acc, Xb, wsh, pinf, npts, lane);
  else if (mode == 4) wave_batch_straight<W>(acc, Xb, wsh, pinf, npts, lane);
  else if (mode == 2 || mode == 3) wave_batch_nofetch<W>(acc, Xb, wsh, pinf, npts, lane, mode == 3);
  else schur_wave_batch<W>(acc, Xb, wsh, pinf, npts, lane);
}
__global__ __launch_bounds__(256) void k_bench(const double* Xg, const int4* pg, int npts, int ntw, int reps,
                                               double* out, unsigned long long* cyc, int mode) {
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
      case 0: run_variant<0>(mode, acc, Xb, wsh, pinf, npts, lane); break;
      case 1: run_variant<1>(mode, acc, Xb, wsh, pinf, npts, lane); break;
      case 2: run_variant<2>(mode, acc, Xb, wsh, pinf, npts, lane); break;
      default: run_variant<3>(mode, acc, Xb, wsh, pinf, npts, lane); break;
    }
  }
  mfma_drain();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int k = 0; k < kSchurTPW; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[tid] = s;
  if (lane == 0) cyc[cw] = t1 - t0;
}
int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int homog = argc > 2 ? atoi(argv[2]) : -1;   // >= 0: every point ends in this window tile
  std::vector<double> X(kSchurXCap);
  for (size_t i = 0; i < X.size(); ++i) X[i] = 1e-3 * (double)((i * 2654435761u) % 1000);
  std::vector<int4> P;
  int xoff = 0, mf = 0, mr = 0;
  for (int t = 0; t < 21; ++t) {
    const int pf = t % 2, span = 6 + (t * 7) % 13;
    const int jhi = homog >= 0 ? homog : (6 * (pf + span) - 1) / 16;
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
  printf("mode %d (homog %d): %d points, %d tile + %d rhs MFMAs per pass (%.1f per wave-point)\n", mode, homog, npts, mf, mr, (mf + mr) / 4.0 / npts);
  hipLaunchKernelGGL(k_bench, dim3(1), dim3(256), 0, 0, Xg, pg, npts, ntw, reps, out, cyc, mode);
  hipLaunchKernelGGL(k_bench, dim3(1), dim3(256), 0, 0, Xg, pg, npts, ntw, reps, out, cyc, mode);
  (void)hipDeviceSynchronize();
  unsigned long long c[8];
  (void)hipMemcpy(c, cyc, 64, hipMemcpyDeviceToHost);
  printf("cycles per point: wave0 %.0f  wave1 %.0f  wave2 %.0f  wave3 %.0f   (MFMA bound %.0f)\n",
         (double)c[0] / (reps * npts), (double)c[1] / (reps * npts), (double)c[2] / (reps * npts),
         (double)c[3] / (reps * npts), 64.0 * (mf + mr) / 4.0 / npts);
  return 0;
}
