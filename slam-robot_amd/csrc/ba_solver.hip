// ba_solver.hip — MI355X-native Levenberg-Marquardt bundle adjustment (the reference's Slam::Run,
// slam.cpp:482-521, which hands the problem to Ceres 1.8 with SPARSE_SCHUR; restated here on gfx950).
//
// One LM iteration = the kernel chain below, enqueued without host synchronisation; the accept/reject
// decision, trust-region update and termination tests run on the device (k_decide), so a solve is a
// stream of identical iterations the host only polls for completion.
//
//   k_linearize    [one wave: rounds of <= 64 observations, lane per observation]  residuals + analytic
//                  Jacobians (HBM sweep), point blocks V,g; camera blocks U,g_c of the co-visibility window
//   k_cam_reduce   deterministic reduce of per-chunk camera partials  -> xchg_cam   (all-reduced)
//   k_cam_finalize FrameDistance terms, cost, gradient test, Jacobi scale (iteration 0), LM diagonal
//   k_schur        [segment of <= 32 points] damped V^-1 (thread per point), P = J_p V^-1 (thread per
//                  observation), Schur blocks -J_c^T P J_p^T J_c (thread per observation pair) into an
//                  LDS window of the segment's camera blocks
//   k_S_reduce     deterministic reduce of the segment windows + blockdiag(U), FrameDistance, damping
//                  -> damped S and rhs (all-reduced across landmark shards)
//   k_cholesky     one workgroup: banded Cholesky of S in an LDS window, back substitution, candidate poses
//   k_point_update back-substitution, model cost change, candidate points, candidate cost
//   k_upd_reduce   reduce of the per-chunk update scalars  -> xchg_upd              (all-reduced)
//   k_decide       Ceres TrustRegionMinimizer / LevenbergMarquardtStrategy bookkeeping
#include <hip/hip_runtime.h>

#include <chrono>
#include <string>
#include <thread>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <numeric>

#include "ba_solver.h"
#include "stager.h"
#include "comm.h"
#include "project_math.h"
#include "schur_tiles.h"

namespace sg {

#ifndef SG_LIN_ATTR
#define SG_LIN_ATTR
#endif

// ------------------------------------------------------------------------------------------------
// small device helpers


// Word copy (8-byte words, grid-stride) between device and mapped host memory.
__global__ __launch_bounds__(256) void k_copy_u64(const unsigned long long* __restrict__ src,
                                                  unsigned long long* __restrict__ dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
// Full-wave sum by DPP (quad perms, half-row and row mirrors) and four readlanes: ~10x faster than the
// ds_bpermute butterfly.  All 64 lanes must be active.  Fixed order, so deterministic; the result is
// wave-uniform.
template <int kCtrl>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), kCtrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), kCtrl, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_dd(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum_full(double v) {
  v += dpp_d<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);   // row_half_mirror
  v += dpp_d<0x140>(v);   // row_mirror: every lane holds its 16-lane row sum
  return (readlane_dd(v, 0) + readlane_dd(v, 16)) + (readlane_dd(v, 32) + readlane_dd(v, 48));
}
// The same butterfly for the maximum (fmax is exact, so any order gives the same bits).  All 64 lanes active.
__device__ __forceinline__ double wave_max_full(double v) {
  v = fmax(v, dpp_d<0xB1>(v));
  v = fmax(v, dpp_d<0x4E>(v));
  v = fmax(v, dpp_d<0x141>(v));
  v = fmax(v, dpp_d<0x140>(v));
  return fmax(fmax(readlane_dd(v, 0), readlane_dd(v, 16)), fmax(readlane_dd(v, 32), readlane_dd(v, 48)));
}
// LDS-only workgroup barrier: waits for this wave's LDS traffic, not for outstanding global loads or
// stores (those may stay in flight across it).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// Sum over aligned groups of 8 lanes by DPP (quad perms, then the half-row mirror pairs lane i with 7 - i):
// every lane of the group gets the group sum, in the same order.  All 64 lanes must be active.
__device__ __forceinline__ double sum8_dpp(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x141>(v);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m));
  return v;
}
// Block reduction in a fixed order (deterministic).  red: LDS scratch of >= nwaves doubles.
template <int NT>
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum_full(v);   // (every thread of the block calls it: all lanes active)
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}
template <int NT>
__device__ __forceinline__ double block_max(double v, double* red) {
  v = wave_max_full(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s = fmax(s, red[i]);
  return s;
}

// Fixed-order workgroup sums of NV values at once: DPP wave sums, one LDS exchange, one barrier; every
// thread gets the totals.  red: LDS of NV * NT / 64 doubles.
template <int NT, int NV>
__device__ __forceinline__ void block_sum_multi(double (&v)[NV], double* red) {
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = wave_sum_full(v[j]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int j = 0; j < NV; ++j) red[w * NV + j] = v[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i * NV + j];
    v[j] = t;
  }
}

// The same sums, for thread 0 only (the large reductions of k_cam_reduce / k_upd_reduce): lane j < NV of wave 0
// sums partial j over the waves in the same fixed order, and thread 0 gathers the totals by v_readlane — every
// thread summing all NV x NT/64 partials held them all in registers at once and spilled (1024-thread, 128-VGPR
// kernels).  Only thread 0's v is meaningful afterwards.
template <int NT, int NV>
__device__ __forceinline__ void block_sum_multi_t0(double (&v)[NV], double* red) {
  static_assert(NV <= 64, "one lane per value");
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = wave_sum_full(v[j]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int j = 0; j < NV; ++j) red[w * NV + j] = v[j];
  __syncthreads();
  if (w == 0) {
    const int j = threadIdx.x < NV ? threadIdx.x : 0;
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i * NV + j];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = readlane_dd(t, k);
  }
}

// packed upper-triangle index of a 6x6 block (a <= c)
__device__ __forceinline__ int u6(int a, int c) { return a * (11 - a) / 2 + c; }
// packed upper-triangle index of a 4x4 block (a <= c)
__device__ __forceinline__ int u4(int a, int c) { return a * (7 - a) / 2 + c; }
// packed index of a window block pair (i <= j < nb)
__device__ __forceinline__ int wp(int i, int j, int nb) { return i * nb - i * (i - 1) / 2 + (j - i); }

// Observation records J (r~ 2 | Jc 12 | Jp 8 | cost, pad) in blocks of 64 observations, element pairs
// interleaved: pair e2 (0..11) of observation o at double2 index ((o >> 6) * 12 + e2) * 64 + (o & 63).  A wave's
// lanes reading (or writing) one element pair of 64 consecutive observations touch one contiguous KiB instead
// of a 16-byte piece of 64 different 192-byte records.
__device__ __forceinline__ size_t jidx2(int o, int e2) { return ((size_t)(o >> 6) * 12 + e2) * 64 + (o & 63); }
__device__ __forceinline__ double2 jload2(const double* J, int o, int e2) {
  return reinterpret_cast<const double2*>(J)[jidx2(o, e2)];
}

// Load the corrected Jacobian of observation o and apply Jacobi scaling.
__device__ __forceinline__ void load_scaled_J(const Dev& d, const double* J, int o, int b, const double* sp,
                                              double* r, double* Jc, double* Jp) {
  double buf[22];
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    const double2 v = jload2(J, o, i);
    buf[2 * i] = v.x;
    buf[2 * i + 1] = v.y;
  }
  r[0] = buf[0];
  r[1] = buf[1];
  if (b >= 0) {
    const double* sc = d.scale_c + 6 * b;
#pragma unroll
    for (int i = 0; i < 12; ++i) Jc[i] = buf[2 + i] * sc[i % 6];
  } else {
#pragma unroll
    for (int i = 0; i < 12; ++i) Jc[i] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) Jp[i] = buf[14 + i] * sp[i % 4];
}

// packed index of a lower-triangular 4x4 (c <= i)
__device__ __forceinline__ int l4(int i, int c) { return i * (i + 1) / 2 + c; }
// 4x4 SPD inverse via LL^T; A and Ainv packed upper (10), L^-1 packed lower (Lo, optional).  Returns false on
// a non-positive pivot.
__device__ __forceinline__ bool inv4_spd(const double* A, double* Ai, double* Lo = nullptr) {
  double L[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) L[i][j] = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double s = A[u4(j, j)];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < j) s -= L[j][k] * L[j][k];
    if (!(s > 0.0)) return false;
    const double ljj = sqrt(s);
    L[j][j] = ljj;
    const double inv = 1.0 / ljj;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i <= j) continue;
      double t = A[u4(j, i)];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < j) t -= L[i][k] * L[j][k];
      L[i][j] = t * inv;
    }
  }
  // Linv (lower)
  double Li[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) Li[i][j] = 0.0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < c) continue;
      double s = (i == c) ? 1.0 : 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k >= c && k < i) s -= L[i][k] * Li[k][c];
      Li[i][c] = s / L[i][i];
    }
  }
  if (Lo)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c <= i; ++c) Lo[l4(i, c)] = Li[i][c];
  // A^-1 = Linv^T Linv
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c < a) continue;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) s += Li[k][a] * Li[k][c];
      Ai[u4(a, c)] = s;
    }
  return true;
}

__device__ __forceinline__ double sym4(const double* A, int a, int c) { return a <= c ? A[u4(a, c)] : A[u4(c, a)]; }

// ------------------------------------------------------------------------------------------------
// k_linearize: the Jacobian sweep.  One LinChunk per single-wave workgroup (independent waves, no workgroup
// barriers, so the chip interleaves one wave's projections with another's loads and stores), one
// observation per lane: each lane evaluates project.h + its analytic Jacobian and the Cauchy corrector and
// stores the corrected 24-double record (r~ 2 | Jc 12 | Jp 8 | cost | pad); its point-block terms
// (V = Jp^T Jp, g = Jp^T r) and camera-block terms (upper Jc^T Jc, Jc^T r) go to LDS accumulators of the
// round's points and of the chunk's camera window.  Only this wave touches its LDS, so the accumulation
// order is fixed (program order, lanes serialised in hardware order).  The next round's observation inputs
// are loaded before this round's projections.
// Wave-local LDS ordering (single-wave workgroups): all of this wave's LDS operations are complete.
__device__ __forceinline__ void lds_fence_wave() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// The chunk's camera partial (the waves' window accumulators summed in wave order) into its cam_slab slot, and
// wave 1's six chunk scalars into wave 0's (sums in wave order, gmax a maximum).  Every thread of the
// workgroup calls it (a workgroup barrier).
template <int kW>
__device__ __forceinline__ void lin_combine_waves(double* slab, double (*camacc_w)[kLinNbMax * kCamV], int ncv,
                                                  double* wscal, int wv, int lane, double& s0, double& s1,
                                                  double& s2, double& s3, double& s4, double& gmax) {
  if (kW == 1) {
    for (int i = lane; i < ncv; i += kLinThreads) slab[i] = camacc_w[0][i];
    return;
  }
  if (wv == 1 && lane == 0) {
    wscal[0] = s0; wscal[1] = s1; wscal[2] = s2; wscal[3] = s3; wscal[4] = s4; wscal[5] = gmax;
  }
  lds_barrier();
  for (int i = threadIdx.x; i < ncv; i += kLinThreads * kW) slab[i] = camacc_w[0][i] + camacc_w[kW - 1][i];
  if (wv == 0) {
    s0 += wscal[0]; s1 += wscal[1]; s2 += wscal[2]; s3 += wscal[3]; s4 += wscal[4];
    gmax = fmax(gmax, wscal[5]);
  }
}

template <int kW>
__global__ __launch_bounds__(kLinThreads * kW) SG_LIN_ATTR void k_linearize(Dev d) {
  const LmState* st = d.st;
  if (st->done || !st->need_lin) return;
  const int cur = st->cur;
  const bool first = st->first != 0;
  const LinChunk ch = d.lchunks[blockIdx.x];
  // per wave (wave w takes every kW-th round of the chunk, see LinChunk):
  __shared__ double pacc_w[kW][kLinPts * 14];         // point blocks of the round: V (10) | g (4)
  __shared__ double camacc_w[kW][kLinNbMax * kCamV];  // camera blocks of the window: upper Jc^T Jc | Jc^T r
  // the rarely-touched per-lane sums (failures, the fixed cost and |X|^2 of iteration 0) live in LDS, one slot
  // per lane, so they hold no registers across the projection (k_linearize's VGPR budget sets its occupancy)
  __shared__ double lsum_w[kW][4][kLinThreads];       // fail, fixed, ffail, xn2
  __shared__ double wscal[8];                         // wave 1's chunk scalars
  const int lane = threadIdx.x & (kLinThreads - 1), wv = threadIdx.x / kLinThreads;
  double* pacc = pacc_w[wv];
  double* camacc = camacc_w[wv];
  double(*lsum)[kLinThreads] = lsum_w[wv];
  // a wide chunk (one point in pieces) runs on wave 0 only
  const int rstep = ch.wide ? 1 : kW, rbeg = ch.r0 + (ch.wide ? 0 : wv);
  const bool active = !ch.wide || wv == 0;
  const double4* X4 = reinterpret_cast<const double4*>(d.X[cur]);
  const int ncv = ch.nb * kCamV;
  for (int i = lane; i < ncv; i += kLinThreads) camacc[i] = 0.0;
  for (int i = lane; i < kLinPts * 14; i += kLinThreads) pacc[i] = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) lsum[k][lane] = 0.0;
  double cost = 0.0, gmax = 0.0;
  // per-observation inputs, software-pipelined one round ahead
  LinRound R{};
  int nobs = 0;
  if (active && rbeg < ch.r1) {
    R = d.lrounds[rbeg];
    nobs = R.o1 - R.o0;
  }
  double2 n_uv = make_double2(0.0, 0.0);
  int n_f = 0, n_p = 0, n_m = 0;
  if (lane < nobs) {
    const int o = R.o0 + lane;
    n_uv = reinterpret_cast<const double2*>(d.obs_pt)[o];
    n_f = d.obs_frame[o];
    n_p = d.obs_pnt[o];
    n_m = d.obs_meta[o];
  }
  lds_fence_wave();
  for (int r = rbeg; active && r < ch.r1; r += rstep) {
    const double2 uv = n_uv;
    const int f = n_f, p = n_p, m = n_m;
    const bool fx = (m & kMetaFixed) != 0;
    const LinRound Rc = R;
    const int nc = nobs;
    if (r + rstep < ch.r1) {
      R = d.lrounds[r + rstep];
      nobs = R.o1 - R.o0;
      if (lane < nobs) {
        const int o = R.o0 + lane;
        n_uv = reinterpret_cast<const double2*>(d.obs_pt)[o];
        n_f = d.obs_frame[o];
        n_p = d.obs_pnt[o];
        n_m = d.obs_meta[o];
      }
    }
    if (lane < nc) {
      const int o = Rc.o0 + lane;
      const bool pf = (m & kMetaPfree) != 0;
      const double4 Xv = X4[p];
      const double X[4] = {Xv.x, Xv.y, Xv.z, Xv.w};
      const double pt[2] = {uv.x, uv.y};
      double rr[2], Jc[12], Jp[8], c;
      const bool ok = LinearizeObservation(d.q[cur] + 4 * f, d.t[cur] + 3 * f, d.k[cur] + 7 * meta_cam(m), X, pt,
                                           d.b, d.inv_b, rr, Jc, Jp, &c);
      double2* Jo = reinterpret_cast<double2*>(d.J[cur]) + jidx2(o, 0);   // pair e2 at Jo[64 e2]
      if (!ok || fx) {
        if (!ok) {
          if (fx) lsum[2][lane] += 1.0;
          else lsum[0][lane] += 1.0;
        } else if (first) {
          lsum[1][lane] += c;
        }
#pragma unroll
        for (int i = 0; i < kJStride / 2; ++i) Jo[64 * i] = make_double2(0.0, 0.0);
      } else {
        cost += c;
        const int b = meta_block(m);
        if (b < 0) {
#pragma unroll
          for (int i = 0; i < 12; ++i) Jc[i] = 0.0;
        } else {
          if (!(m & kMetaRot)) { Jc[0] = Jc[1] = Jc[2] = Jc[6] = Jc[7] = Jc[8] = 0.0; }
          if (!(m & kMetaTrans)) { Jc[3] = Jc[4] = Jc[5] = Jc[9] = Jc[10] = Jc[11] = 0.0; }
        }
        if (!pf) {
#pragma unroll
          for (int i = 0; i < 8; ++i) Jp[i] = 0.0;
        }
        Jo[0] = make_double2(rr[0], rr[1]);
#pragma unroll
        for (int i = 0; i < 6; ++i) Jo[64 * (1 + i)] = make_double2(Jc[2 * i], Jc[2 * i + 1]);
#pragma unroll
        for (int i = 0; i < 4; ++i) Jo[64 * (7 + i)] = make_double2(Jp[2 * i], Jp[2 * i + 1]);
        Jo[64 * 11] = make_double2(c, 0.0);
        if (pf) {
          double* pa = pacc + (p - Rc.p0) * 14;
#pragma unroll
          for (int a = 0; a < 4; ++a) {
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
              if (cc >= a) atomicAdd(pa + u4(a, cc), Jp[a] * Jp[cc] + Jp[4 + a] * Jp[4 + cc]);
            atomicAdd(pa + 10 + a, Jp[a] * rr[0] + Jp[4 + a] * rr[1]);
          }
        }
        if (b >= 0) {
          // separate paths: a pointer that may be LDS or global would make these flat atomics
          auto add_cam = [&](double* dst) {
#pragma unroll
            for (int a = 0; a < 6; ++a) {
#pragma unroll
              for (int cc = 0; cc < 6; ++cc)
                if (cc >= a) atomicAdd(dst + u6(a, cc), Jc[a] * Jc[cc] + Jc[6 + a] * Jc[6 + cc]);
              atomicAdd(dst + 21 + a, Jc[a] * rr[0] + Jc[6 + a] * rr[1]);
            }
          };
          if (ch.wide) add_cam(d.cam_wide[cur] + (size_t)b * kCamV);
          else add_cam(camacc + (b - ch.b_lo) * kCamV);
        }
      }
    }
    // point blocks of the round's (whole) points; a wide chunk's one point after its last piece
    if (!ch.wide || r + 1 == ch.r1) {
      lds_fence_wave();
      const int np = Rc.p1 - Rc.p0;
      if (lane < np) {
        const int pp = Rc.p0 + lane;
        double* pa = pacc + lane * 14;
        double V[10], g[4];
#pragma unroll
        for (int i = 0; i < 10; ++i) V[i] = pa[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) g[i] = pa[10 + i];
#pragma unroll
        for (int i = 0; i < 14; ++i) pa[i] = 0.0;
        const bool pf = d.pfree[pp] != 0;
        double2* Vd = reinterpret_cast<double2*>(d.V[cur] + 10 * (size_t)pp);
#pragma unroll
        for (int k = 0; k < 5; ++k) Vd[k] = make_double2(V[2 * k], V[2 * k + 1]);
        reinterpret_cast<double4*>(d.g[cur])[pp] = make_double4(g[0], g[1], g[2], g[3]);
        if (pf) {
          gmax = fmax(gmax, fmax(fmax(fabs(g[0]), fabs(g[1])), fmax(fabs(g[2]), fabs(g[3]))));
          if (first) {
            reinterpret_cast<double4*>(d.scale_p)[pp] =
                make_double4(1.0 / (1.0 + sqrt(V[0])), 1.0 / (1.0 + sqrt(V[4])), 1.0 / (1.0 + sqrt(V[7])),
                             1.0 / (1.0 + sqrt(V[9])));
            const double4 Xv = X4[pp];
            lsum[3][lane] += Xv.x * Xv.x + Xv.y * Xv.y + Xv.z * Xv.z + Xv.w * Xv.w;
          }
        } else if (first) {
          reinterpret_cast<double4*>(d.scale_p)[pp] = make_double4(1.0, 1.0, 1.0, 1.0);
        }
      }
      lds_fence_wave();
    }
  }
  lds_fence_wave();
  cost = wave_sum_full(cost);
  double fail = wave_sum_full(lsum[0][lane]);
  double fixed = wave_sum_full(lsum[1][lane]);
  double ffail = wave_sum_full(lsum[2][lane]);
  double xn2 = wave_sum_full(lsum[3][lane]);
  gmax = wave_max_full(gmax);
  lin_combine_waves<kW>(d.cam_slab[cur] + ch.cam_off, camacc_w, ncv, wscal, wv, lane, cost, fail, fixed, ffail,
                        xn2, gmax);
  if (wv == 0 && lane == 0) {
    double* sc = d.lin_scal[cur] + blockIdx.x;   // structure of arrays: slot j at [j * nlin + chunk]
    const size_t ns = d.nlin;
    sc[kCost * ns] = cost;
    sc[kFail * ns] = fail;
    sc[kFixed * ns] = fixed;
    sc[kFixedFail * ns] = ffail;
    sc[kXnorm2 * ns] = xn2;
    sc[kGmax * ns] = gmax;
  }
}

// ------------------------------------------------------------------------------------------------
// k_cam_reduce: deterministic sum of the per-chunk camera partials (+ wide-chunk atomics).  One workgroup
// per camera block: kCamSlices slices x 27 elements, each slice summing every kCamSlices-th partial of the
// block's list, the slices combined in slice order; the last workgroup reduces the chunk scalars.
constexpr int kCamSlices = 32;
constexpr int kRedThreads = 1024;   // >= kCamSlices * kCamV
__device__ void upd_reduce_body(const Dev& d, int fuse);

// mode 0: the current slot's partials (after a solve's first k_linearize, or after k_linearize in the two-pass
//         chain), into xchg_cam / xcam_loc; a step that did not linearize (need_lin = 0) leaves them, and with
//         landmark shards copies this rank's blocks into the all-reduce buffer again;
// mode 1: speculative chain, right after k_update_lin: the candidate slot's partials into xchg_cand (the decision
//         that follows copies them to the current blocks if it accepts the step), and block NB + 1 reduces the
//         update scalars (k_upd_reduce without the decision).  Nothing here writes LmState, so every block reads
//         the same slot.
// mode 2: mode 1 with the decision in block NB + 1 (one rank): the step is decided here, so every block takes the
//         candidate slot from LmState::spec_slot (written by k_update_lin, unchanged by the decision), not from cur.
__global__ __launch_bounds__(kRedThreads) void k_cam_reduce(Dev d, int mode) {
  const LmState* st = d.st;
  if (mode >= 1 && (int)blockIdx.x == d.NB + 1) {
    upd_reduce_body(d, mode == 2 ? 1 : 0);
    return;
  }
  if (st->done) return;
  const int tid = threadIdx.x;
  const int nv = d.NB * kCamV;
  const int nx = nv + kXNum + d.nranks;
  if (mode == 0 && !st->need_lin) {
    // no new linearization: the shards' camera-block all-reduce sums this rank's current blocks again
    if (d.nranks > 1 && blockIdx.x == 0)
      for (int i = tid; i < nx; i += blockDim.x) d.xchg_cam[i] = d.xcam_loc[i];
    return;
  }
  const int cur = mode >= 1 ? st->spec_slot : st->cur;
  double* dst = mode >= 1 ? d.xchg_cand : d.xchg_cam;
  double* dst2 = mode >= 1 ? d.xchg_cand : d.xcam_loc;
  if ((int)blockIdx.x < d.NB) {
    const int b = blockIdx.x;
    __shared__ double part[kCamSlices][kCamV];
    const int e = tid % kCamV, sl = tid / kCamV;
    if (sl < kCamSlices) {
      const int j0 = d.cam_loff[b], j1 = d.cam_loff[b + 1];
      double acc = 0.0;
#ifndef SG_CAM_RED_U
#define SG_CAM_RED_U 16
#endif
      constexpr int kU = SG_CAM_RED_U;   // offsets, then partials, kU at a time in flight (one round of each at C2)
      for (int jb = j0 + sl; jb < j1; jb += kU * kCamSlices) {
        int ix[kU];
        double v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) ix[u] = d.cam_lidx[jb + u * kCamSlices < j1 ? jb + u * kCamSlices : 0];   // unconditional
#pragma unroll
        for (int u = 0; u < kU; ++u) v[u] = d.cam_slab[cur][ix[u] + e];
#pragma unroll
        for (int u = 0; u < kU; ++u)
          if (jb + u * kCamSlices < j1) acc += v[u];
      }
      part[sl][e] = acc;
    }
    __syncthreads();
    if (tid < kCamV) {
      const int i = b * kCamV + tid;
      double s = d.cam_wide[cur][i];
      // (speculative mode: kept, a re-reduce after a rejected step reads it again; k_S_reduce clears the
      // candidate slot before k_update_lin accumulates into it)
      if (!d.spec) d.cam_wide[cur][i] = 0.0;
#pragma unroll
      for (int k = 0; k < kCamSlices; ++k) s += part[k][tid];
      dst[i] = s;    // summed over the shards (camera-block all-reduce) or left as this rank's
      dst2[i] = s;   // this rank's own (k_S_reduce's local assembly, k_cam_finalize mode 1)
    }
    return;
  }
  // scalars: thread t sums chunks t, t + 1024, ... (two chunks' loads in flight), then a fixed-order
  // workgroup tree
  __shared__ double red[kRedThreads / 64 * kXNum];
  __shared__ double redm[kRedThreads / 64];
  double v[kXNum] = {0, 0, 0, 0, 0};
  double gm = 0.0;
#ifndef SG_SCAL_RED_U
#define SG_SCAL_RED_U 2
#endif
  constexpr int kScalU = SG_SCAL_RED_U;   // chunks' loads in flight per thread (8 measured slower)
  for (int c0 = tid; c0 < d.nlin; c0 += kScalU * kRedThreads) {
    double t[kScalU][kXNum + 1];
#pragma unroll
    for (int u = 0; u < kScalU; ++u) {
      const int c = c0 + u * kRedThreads;
      const double* sc = d.lin_scal[cur] + (c < d.nlin ? c : 0);   // coalesced: slot j at [j * nlin + chunk]
      const size_t ns = d.nlin;
      t[u][kXCost] = sc[kCost * ns];
      t[u][kXFail] = sc[kFail * ns];
      t[u][kXFixed] = sc[kFixed * ns];
      t[u][kXFixedFail] = sc[kFixedFail * ns];
      t[u][kXXnorm2] = sc[kXnorm2 * ns];
      t[u][kXNum] = sc[kGmax * ns];
    }
#pragma unroll
    for (int u = 0; u < kScalU; ++u)
      if (c0 + u * kRedThreads < d.nlin) {
#pragma unroll
        for (int j = 0; j < kXNum; ++j) v[j] += t[u][j];
        gm = fmax(gm, t[u][kXNum]);
      }
  }
  block_sum_multi_t0<kRedThreads, kXNum>(v, red);
  gm = block_max<kRedThreads>(gm, redm);
  if (tid == 0) {
#pragma unroll
    for (int j = 0; j < kXNum; ++j) dst[nv + j] = dst2[nv + j] = v[j];
    // max |g| travels in the same sum all-reduce: one slot per rank, zeros in the others' slots
    for (int r = 0; r < d.nranks; ++r) dst[nv + kXNum + r] = dst2[nv + kXNum + r] = (r == d.rank) ? gm : 0.0;
  }
}

// ------------------------------------------------------------------------------------------------
// k_cam_finalize: one workgroup.  FrameDistance blocks (slam.cpp:86-105), total cost, gradient
// max-norm, Jacobi scale (iteration 0), pending iteration push, max-iteration test, LM diagonal.
// A single workgroup's latency chain: the FrameDistance Jacobians and the camera gradient / diagonal stay in
// LDS for the passes that re-read them (global copies are still written for k_S_reduce), and the block
// pass's exchange-buffer operands are loaded before the FrameDistance pass.
constexpr int kFinFdSh = 256;    // FrameDistance residuals held in LDS (more: re-read from global)
constexpr int kFinNSh = 1536;    // frame columns held in LDS (more: re-read from global)
// Ceres TrustRegionMinimizer bookkeeping of a linearized iteration (thread 0, on a register copy of LmState):
// iteration 0's cost / fixed cost / failures / gradient tolerance, or a later iteration's push.
__device__ __forceinline__ void fin_push(LmState& s0, bool first, double cost, double gmax, const double* xs,
                                         double xn2c) {
  if (first) {
    s0.fixed_cost = xs[kXFixed];
    if (xs[kXFixedFail] > 0.0) {
      s0.done = 1; s0.ok = 0; s0.termination = SG_DID_NOT_RUN;
    } else if (xs[kXFail] > 0.0) {
      s0.done = 1; s0.ok = 0; s0.termination = SG_NUMERICAL_FAILURE;
    } else {
      s0.cost = cost;
      s0.initial_cost = cost + s0.fixed_cost;
      s0.abs_gtol = s0.gtol * gmax;
      s0.pushed = 1;
      s0.min_pushed_cost = cost;
      s0.x_norm = sqrt(xs[kXXnorm2] + xn2c);
      if (gmax <= s0.abs_gtol && !s0.disable_term) {
        s0.done = 1; s0.ok = 1; s0.termination = SG_GRADIENT_TOLERANCE;
      }
    }
    s0.first = 0;
  } else {
    if (xs[kXFail] > 0.0) {
      s0.done = 1; s0.ok = 0; s0.termination = SG_NUMERICAL_FAILURE;
    } else {
      s0.cost = cost;
      if (!s0.disable_term && gmax <= s0.abs_gtol) {
        s0.done = 1; s0.ok = 1; s0.termination = SG_GRADIENT_TOLERANCE;
      } else if (!s0.disable_term && s0.radius < s0.min_radius) {
        s0.done = 1; s0.ok = 1; s0.termination = SG_PARAMETER_TOLERANCE;
      } else {
        s0.pushed += 1;
        s0.min_pushed_cost = fmin(s0.min_pushed_cost, cost);
      }
    }
  }
  s0.need_lin = 0;
}

// The max-iteration tests and the LM iteration count (every iteration, linearized or not).
__device__ __forceinline__ void fin_count(LmState& s0) {
  if (!s0.done) {
    if (!s0.disable_term && s0.pushed - 1 >= s0.max_iter) {
      s0.done = 1; s0.ok = 1; s0.termination = SG_NO_CONVERGENCE;
    } else if (s0.disable_term && s0.lm_iters >= s0.max_iter) {
      s0.done = 1; s0.ok = 1; s0.termination = SG_NO_CONVERGENCE;
    }
  }
  if (!s0.done) s0.lm_iters += 1;
}

// mode 0: everything, on the summed camera blocks (one rank, or landmark shards after the camera-block
//         all-reduce: a solve's first iteration, which fixes the Jacobi scale);
// mode 1: landmark shards after the first iteration, before the merged exchange — this rank's camera gradient
//         and diagonal (its own blocks; the FrameDistance terms on rank 0) for k_S_reduce's local assembly and
//         into the exchange tail with the cost scalars; no bookkeeping;
// mode 2: after the merged exchange (every rank, identically): the bookkeeping on the summed tail, the LM
//         diagonal, and the damping D^2 / radius added to the summed S (k_S_reduce's local assembly leaves it out).
// decide 1: merged shards after the update-scalar all-reduce: thread 0 first takes the pending step's decision
// (decide_step, as k_decide) and, when it accepts, the candidate's camera blocks and scalars (k_cam_reduce
// mode 1, xchg_cand) become the current ones — so no separate decision launch;
// decide 2: one rank: the decision was taken by k_cam_reduce mode 2; an accepted step's candidate blocks are
// taken here (LmState::accepted).
__device__ void decide_step(LmState& s, const double* u, const double* c);
// LDS of the finalize pass: its own in k_cam_finalize, carved from k_schur's operand buffer when a k_schur launch
// runs it in one extra workgroup (k_schur's fin).
struct FinLds {
  double *red, *fdcost, *fdJs, *fdrs, *gsh, *dgsh, *scsh;
  int *dsh, *done_sh;
  static constexpr int kDoubles = 8 + 256 + 7 * kFinFdSh + 3 * kFinNSh + 4;
  __device__ static FinLds carve(double* p) {
    FinLds L;
    L.red = p;
    L.fdcost = p + 8;
    L.fdJs = L.fdcost + 256;
    L.fdrs = L.fdJs + 6 * kFinFdSh;
    L.gsh = L.fdrs + kFinFdSh;
    L.dgsh = L.gsh + kFinNSh;
    L.scsh = L.dgsh + kFinNSh;
    L.dsh = reinterpret_cast<int*>(L.scsh + kFinNSh);
    L.done_sh = L.dsh + 4;
    return L;
  }
};

// The pass on the first 256 threads of the workgroup (the others only meet the barriers: k_schur's
// workgroups are larger).
__device__ __forceinline__ void cam_finalize_body(const Dev& d, int mode, int decide, const FinLds& L) {
  LmState* st = d.st;
  double* red = L.red;      // >= 8 (one slot per wave of a 512-thread workgroup)
  int* dsh = L.dsh;         // after the decision: cur, need_lin, done, accepted
  double* fdcost = L.fdcost;
  double* fdJs = L.fdJs;
  double* fdrs = L.fdrs;
  double* gsh = L.gsh;
  double* dgsh = L.dgsh;
  double* scsh = L.scsh;
  int& done_sh = *L.done_sh;
  const int tid = threadIdx.x;
  const bool act = tid < 256;
  const int nv = d.NB * kCamV;
  const int nf = 6 * d.NB;
  const bool fd_lds = d.D <= kFinFdSh, n_lds = nf <= kFinNSh;
  // exchange tail (modes 1, 2): camera gradient [nf] | camera diagonal [nf] | scalars [kXNum] | per-rank max |g|
  // [nranks] | FrameDistance cost
  double* tg = d.xtail;
  double* tdg = d.xtail + nf;
  double* txs = d.xtail + 2 * nf;
  const double* U0 = mode == 1 ? d.xcam_loc : d.xchg_cam;
  // block pass operands of block tid (the common case NB <= 256) and the first FrameDistance pair: their
  // loads go out beside LmState's (see k_S_reduce) and stay in flight during the FrameDistance pass
  double Ug[6], Ud[6], Ugc[6], Udc[6];
  int e0 = 0, e1 = 0;
  const int b0 = tid < d.NB ? tid : 0;
  if (mode != 2) {
    const double* U = U0 + (size_t)b0 * kCamV;
    const double* Uc = d.xchg_cand + (size_t)b0 * kCamV;   // (read only when a decision accepts)
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      Ug[a] = U[21 + a];
      Ud[a] = U[u6(a, a)];
      if (decide) {
        Ugc[a] = Uc[21 + a];
        Udc[a] = Uc[u6(a, a)];
      }
    }
    e0 = d.fd_boff[b0];
    e1 = d.fd_boff[b0 + 1];
  }
  const int dd0 = tid < d.D ? tid : 0;
  // thread 0 runs the minimizer bookkeeping on a register copy of LmState (loaded beside the prefetches, written
  // back once): no chain of dependent global round trips through st->
  LmState s0;
  if (tid == 0) s0 = *st;
  const int fa0 = d.D > 0 ? d.fd_a[dd0] : 0, fb0 = d.D > 0 ? d.fd_b[dd0] : 0;
  // read once, before thread 0 updates them below (no other thread re-reads LmState flags afterwards)
  const bool first = st->first, jacobi = st->jacobi;
  int cur;
  bool lin;
  if (decide) {
    if (tid == 0) {
      int acc = 0;
      if (decide == 1 && !s0.done) {
        const int c0 = s0.cur;
        decide_step(s0, d.xchg_upd, d.xchg_chol);
        acc = s0.cur != c0;
      } else if (decide == 2) {
        acc = s0.accepted;
      }
      s0.accepted = 0;
      dsh[0] = s0.cur;
      dsh[1] = s0.need_lin;
      dsh[2] = s0.done;
      dsh[3] = acc;
    }
    __syncthreads();
    cur = dsh[0];
    lin = dsh[1];
    if (dsh[2]) {
      if (tid == 0) *st = s0;
      return;
    }
    if (dsh[3]) {   // accepted: the candidate's blocks and scalars are the current ones from here on
      const int nx = nv + kXNum + d.nranks;
      for (int i = tid; act && i < nx; i += 256) {
        const double v = d.xchg_cand[i];
        d.xchg_cam[i] = v;
        d.xcam_loc[i] = v;
      }
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        Ug[a] = Ugc[a];
        Ud[a] = Udc[a];
      }
      __syncthreads();
    }
  } else {
    cur = st->cur;
    lin = st->need_lin;
    if (st->done) return;
  }
  if (mode == 2) {
    if (lin) {
      // gradient max-norm over the free camera columns of the summed gradient, and the per-rank point maxima
      double gm = 0.0;
      for (int f = tid; act && f < d.F; f += 256) {
        const int b = d.frame_block[f];
        if (b < 0) continue;
        if (d.rot_free[f])
          for (int a = 0; a < 3; ++a) gm = fmax(gm, fabs(tg[6 * b + a]));
        if (d.trans_free[f])
          for (int a = 3; a < 6; ++a) gm = fmax(gm, fabs(tg[6 * b + a]));
      }
      gm = block_max<256>(gm, red);
      if (tid == 0) {
        double gmax = gm;
        for (int r = 0; r < d.nranks; ++r) gmax = fmax(gmax, txs[kXNum + r]);
        fin_push(s0, false, txs[kXCost] + txs[kXNum + d.nranks], gmax, txs, 0.0);
      }
    }
    __syncthreads();
    if (tid == 0) {
      fin_count(s0);
      done_sh = s0.done;
      *st = s0;
    }
    __syncthreads();
    if (done_sh) return;
    const double radius = st->radius;
    const bool reuse = st->reuse_diag;
    for (int i = tid; act && i < d.n; i += 256) {
      double dg;
      if (!reuse) {
        const double s = d.scale_c[i];
        dg = fmin(fmax(s * s * tdg[i], st->min_diag), st->max_diag);
        d.diag_c[i] = dg;
      } else {
        dg = d.diag_c[i];
      }
      d.S[(size_t)i * d.n + i] += dg / radius;
    }
    return;
  }
  // mode 1: the FrameDistance terms enter the exchange on rank 0 only; every rank still evaluates them (fd_r,
  // fd_J, fd_X, fd_D: the Cholesky's candidate pass takes its FrameDistance model term from them, identically
  // on every rank)
  const bool fd_here = mode == 0 || d.rank == 0;
  if (lin) {
    // FrameDistance residuals at x[cur]
    double myfd = 0.0;
    for (int dd = tid; act && dd < d.D; dd += 256) {
      const int fa = dd == tid ? fa0 : d.fd_a[dd], fb = dd == tid ? fb0 : d.fd_b[dd];
      const double* ta = d.t[cur] + 3 * fa;
      const double* tb = d.t[cur] + 3 * fb;
      const double e0_ = ta[0] - tb[0], e1_ = ta[1] - tb[1], e2_ = ta[2] - tb[2];
      const double dist = sqrt(e0_ * e0_ + e1_ * e1_ + e2_ * e2_);
      const double r = 0.1 * (dist - d.fd_target);
      double rho0, rho1;
      Cauchy(r * r, d.fd_b2, d.fd_inv_b2, &rho0, &rho1);
      myfd += 0.5 * rho0;
      const double sr = sqrt(rho1);
      d.fd_r[dd] = sr * r;
      const double gsc = sr * 0.1 / dist;
      const double ga[3] = {gsc * e0_, gsc * e1_, gsc * e2_};
      const bool af = d.trans_free[fa] && d.frame_block[fa] >= 0;
      const bool bf = d.trans_free[fb] && d.frame_block[fb] >= 0;
      double Jd[6];
      for (int j = 0; j < 3; ++j) {
        Jd[j] = af ? ga[j] : 0.0;
        Jd[3 + j] = bf ? -ga[j] : 0.0;
      }
      for (int j = 0; j < 6; ++j) d.fd_J[6 * dd + j] = Jd[j];
      if (fd_lds) {
        fdrs[dd] = sr * r;
        for (int j = 0; j < 6; ++j) fdJs[6 * dd + j] = Jd[j];
      }
      double* Xd = d.fd_X + 9 * dd;
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Xd[3 * i + j] = Jd[i] * Jd[3 + j];
    }
    // FrameDistance cost: DPP wave sums, then the four waves in order (the barrier also publishes the LDS
    // FD terms for the block pass)
    {
      const double w = wave_sum_full(myfd);
      if ((tid & 63) == 0) fdcost[tid >> 6] = w;
    }
    __syncthreads();
    const double fd_total = (fdcost[0] + fdcost[1]) + (fdcost[2] + fdcost[3]);
    // per camera block: gradient, diag, FD diagonal block
    double gm = 0.0, xn2c = 0.0;
    for (int b = tid; act && b < d.NB; b += 256) {
      if (b != tid) {   // NB > 256: operands not prefetched
        const double* U = U0 + (size_t)b * kCamV;
        for (int a = 0; a < 6; ++a) {
          Ug[a] = U[21 + a];
          Ud[a] = U[u6(a, a)];
        }
        e0 = d.fd_boff[b];
        e1 = d.fd_boff[b + 1];
      }
      double fdD[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      double gfd[3] = {0, 0, 0};
      for (int e = e0; e < e1; ++e) {
        const int dd = d.fd_bidx[e] >> 1, side = d.fd_bidx[e] & 1;
        const double* Jd = fd_lds ? fdJs + 6 * dd + 3 * side : d.fd_J + 6 * dd + 3 * side;
        const double rr = fd_lds ? fdrs[dd] : d.fd_r[dd];
        for (int i = 0; i < 3; ++i) {
          gfd[i] += Jd[i] * rr;
          for (int j = 0; j < 3; ++j) fdD[3 * i + j] += Jd[i] * Jd[j];
        }
      }
      for (int i = 0; i < 9; ++i) d.fd_D[9 * b + i] = fdD[i];
      for (int a = 0; a < 6; ++a) {
        const double gg = Ug[a] + ((fd_here && a >= 3) ? gfd[a - 3] : 0.0);
        const double dg = Ud[a] + ((fd_here && a >= 3) ? fdD[4 * (a - 3)] : 0.0);
        d.camg[6 * b + a] = gg;
        d.camdiag[6 * b + a] = dg;
        if (mode == 1) {
          tg[6 * b + a] = gg;
          tdg[6 * b + a] = dg;
        }
        if (n_lds) {
          gsh[6 * b + a] = gg;
          dgsh[6 * b + a] = dg;
        }
      }
    }
    if (mode == 1) {
      // this rank's cost scalars and max |g| slots, and the FrameDistance cost (rank 0), into the tail
      if (tid < kXNum + d.nranks) txs[tid] = d.xcam_loc[nv + tid];
      if (tid == 0) {
        txs[kXNum + d.nranks] = fd_here ? fd_total : 0.0;
        if (decide) *st = s0;   // the decision taken above (the bookkeeping follows the exchange, mode 2)
      }
      return;
    }
    __syncthreads();
    // gradient max-norm over free camera columns; camera part of |x| at iteration 0
    for (int f = tid; act && f < d.F; f += 256) {
      const int b = d.frame_block[f];
      if (b < 0) continue;
      // (the value is selected, not the pointer: an LDS-or-global pointer compiles to flat accesses)
      auto cg = [&](int i) { return n_lds ? gsh[i] : d.camg[i]; };
      if (d.rot_free[f])
        for (int a = 0; a < 3; ++a) gm = fmax(gm, fabs(cg(6 * b + a)));
      if (d.trans_free[f])
        for (int a = 3; a < 6; ++a) gm = fmax(gm, fabs(cg(6 * b + a)));
      if (first) {
        if (d.rot_free[f])
          for (int a = 0; a < 4; ++a) xn2c += d.q[cur][4 * f + a] * d.q[cur][4 * f + a];
        if (d.trans_free[f])
          for (int a = 0; a < 3; ++a) xn2c += d.t[cur][3 * f + a] * d.t[cur][3 * f + a];
      }
    }
    gm = block_max<256>(gm, red);
    xn2c = block_sum<256>(xn2c, red);
    if (first) {
      for (int i = tid; act && i < d.n; i += 256) {
        const double cd = (n_lds && i < nf) ? dgsh[i] : d.camdiag[i];
        const double sc = jacobi ? 1.0 / (1.0 + sqrt(cd)) : 1.0;
        d.scale_c[i] = sc;
        if (n_lds && i < nf) scsh[i] = sc;
      }
    }
    if (tid == 0) {
      const double* xs = d.xchg_cam + nv;
      double gmax = gm;
      for (int r = 0; r < d.nranks; ++r) gmax = fmax(gmax, xs[kXNum + r]);
      fin_push(s0, first, xs[kXCost] + fd_total, gmax, xs, xn2c);
    }
  }
  if (mode == 1) {
    // not linearized (a rejected step): the tail is not read after the exchange; keep it finite
    for (int i = tid; act && i < 2 * nf + kXNum + d.nranks + 1; i += 256) d.xtail[i] = 0.0;
    if (decide && tid == 0) *st = s0;
    return;
  }
  __syncthreads();
  if (tid == 0) {
    fin_count(s0);
    done_sh = s0.done;
    *st = s0;
  }
  __syncthreads();
  if (done_sh) return;
  if (!st->reuse_diag)
    for (int i = tid; act && i < d.n; i += 256) {
      const bool sh = lin && n_lds && i < nf;   // written above in this launch
      const double s = (sh && first) ? scsh[i] : d.scale_c[i];
      const double cd = sh ? dgsh[i] : d.camdiag[i];
      d.diag_c[i] = fmin(fmax(s * s * cd, st->min_diag), st->max_diag);
    }
}

__global__ __launch_bounds__(256) void k_cam_finalize(Dev d, int mode, int decide) {
  __shared__ double lds[FinLds::kDoubles];
  cam_finalize_body(d, mode, decide, FinLds::carve(lds));
}

// ------------------------------------------------------------------------------------------------
// k_schur: the point elimination S -= W V~^-1 W^T and rhs -= W V~^-1 g~, as batched rank-4 updates on the
// matrix cores.
//
// For a free point p with damped, scaled block V~ = L L^T, whiten its camera Jacobians per block b of its
// span:  E_{p,b} = L^-1 sum_{o of p in b} J~p,o^T J~c,o  (4 x 6; zero for a block it does not observe).
// Then its Schur term over every block pair of its span is E_p^T E_p with E_p = [E_{p,b}]_b (4 x 6 span), and
// its rhs term is E_p^T w_p with w_p = L^-1 g~ — one v_mfma_f64_16x16x4f64 per 16x16 tile of S the point
// touches (K = 4: one point per MFMA).  Two observations of p in one block simply sum into one E_{p,b}.
//
// One workgroup (4 waves) per segment: consecutive points (device order: by first block) whose columns fit
// a window of kSchurTW tiles of S.  The window's upper tiles stay in MFMA accumulators for the whole
// segment — wave w owns tiles u = w + 4 s (column-major upper order) — so every tile of a segment is
// written once, summed in point order (bitwise reproducible).  The segment streams through LDS in batches:
//   1. thread per point: V~, L^-1, V~^-1 and t = V~^-1 g~ (for k_point_update), w = L^-1 g~;
//   2. thread per cell (point, block of its span): E_{p,b} and its rhs term E_{p,b}^T w_p;
//   3. every wave walks the batch's points: operands X_j[lane i + 16 k] = E_p[k][16 j + i] read straight
//      from the cells, one MFMA per owned tile inside the point's span; the rhs threads (6 per block of the
//      segment) add the cells' rhs terms.
// Points spanning more than kSegNbMax blocks take k_schur_wide (observation pairs, global atomics).

__device__ __forceinline__ void load_Jc_scaled(const Dev& d, const double* J, int o, int b, double* Jc) {
  const double* sc = d.scale_c + 6 * b;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double2 v = jload2(J, o, 1 + i);   // (pair 0: r)
    Jc[2 * i] = v.x * sc[(2 * i) % 6];
    Jc[2 * i + 1] = v.y * sc[(2 * i + 1) % 6];
  }
}
__device__ __forceinline__ void load_Jp_scaled(const double* J, int o, const double4& s4, double* Jp) {
  const double sp[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double2 v = jload2(J, o, 7 + i);   // (pairs 0-6: r, Jc)
    Jp[2 * i] = v.x * sp[(2 * i) % 4];
    Jp[2 * i + 1] = v.y * sp[(2 * i + 1) % 4];
  }
}

// Damped, scaled point block of point p: V~ = S V S + D^2 / radius (D^2 = clamped diag(S V S), refreshed
// unless the step reuses it), its inverse and L^-1 (V~ = L L^T), t = V~^-1 g~, w = L^-1 g~; Vinv, tp and
// diag_p go to global memory for k_point_update.  Returns false when V~ is not positive definite (Vi, Li NaN).
__device__ __forceinline__ bool point_block(const Dev& d, const LmState* st, int p, double* Vi, double* Li,
                                            double* w) {
  const double* Vp = d.V[st->cur] + 10 * (size_t)p;
  double V[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) V[i] = Vp[i];
  const double4 s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
  const double sp[4] = {s4.x, s4.y, s4.z, s4.w};
  const double4 g4 = reinterpret_cast<const double4*>(d.g[st->cur])[p];
  const double gs[4] = {g4.x * sp[0], g4.y * sp[1], g4.z * sp[2], g4.w * sp[3]};
  double dp[4];
  if (!st->reuse_diag) {
#pragma unroll
    for (int a = 0; a < 4; ++a) dp[a] = fmin(fmax(sp[a] * sp[a] * V[u4(a, a)], st->min_diag), st->max_diag);
    reinterpret_cast<double4*>(d.diag_p)[p] = make_double4(dp[0], dp[1], dp[2], dp[3]);
  } else {
    const double4 d4 = reinterpret_cast<const double4*>(d.diag_p)[p];
    dp[0] = d4.x; dp[1] = d4.y; dp[2] = d4.z; dp[3] = d4.w;
  }
  const double radius = st->radius;
  double Vt[10];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c >= a) Vt[u4(a, c)] = sp[a] * V[u4(a, c)] * sp[c] + (a == c ? dp[a] / radius : 0.0);
  const bool ok = inv4_spd(Vt, Vi, Li);
  if (!ok) {
#pragma unroll
    for (int i = 0; i < 10; ++i) Vi[i] = Li[i] = NAN;
  }
  double tp[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) s += sym4(Vi, a, c) * gs[c];
    tp[a] = s;
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c <= a; ++c) s += Li[l4(a, c)] * gs[c];
    w[a] = s;
  }
  double* Vo = d.Vinv + 10 * (size_t)p;
#pragma unroll
  for (int i = 0; i < 10; ++i) Vo[i] = Vi[i];
  reinterpret_cast<double4*>(d.tp)[p] = make_double4(tp[0], tp[1], tp[2], tp[3]);
  return ok;
}

// The segment's batches run as a software pipeline over three wave groups, one LDS barrier per step:
//   cell waves (kSchurCellWaves), step s: the operand tiles of batch s (buffer s % 2);
//   the point wave, step s: the point blocks of batch s + 1 (point slot (s + 1) % 3);
//   MFMA waves (kSchurCWaves), step s: batch s - 1 (buffer (s - 1) % 2, point slot (s - 1) % 3).
// The groups run separate loops with the same barrier count, so the accumulators are not live elsewhere.
struct SchurLds {
  double X[2][kSchurXCap + 64 * kSchurTW];   // operand tiles of the batch's points; padding for over-reads
  double L[3][kSchurBatchPts * 10];          // L^-1 of the batch's points
  double w[3][kSchurBatchPts * 4];           // w = L^-1 g~
  int4 pinf[3][kSchurBatchPts];              // first block, span, operand offset, last window tile (jhi)
  int2 pob[3][kSchurBatchPts];               // observation of its first block (-1: cell records), first cell
  uint8_t cmap[3][kSchurBatchCells];         // batch-local cell -> point
  double red[kSchurThreads / 64];
};

// Point wave, thread t < npts of batch B: its point block, table entries and cell map.
__device__ __forceinline__ double schur_points(const Dev& d, const LmState* st, const SchurBatch& B, int t,
                                               double* Lsh, double* wsh, int4* pinf, int2* pob, uint8_t* cmap) {
  if (t >= B.p1 - B.p0) return 0.0;
  const int p = B.p0 + t;
  const int2 pi = d.pinfo[p];
  const int4 pm = d.pmx[p];   // operand offset, jhi, observation of the first block (-1), first cell
  int span = pi.y & 0xff, jhi = pm.y;
  double fail = 0.0;
  if (d.pfree[p]) {
    double Vi[10], Li[10], w[4];
    if (!point_block(d, st, p, Vi, Li, w)) fail = 1.0;
#pragma unroll
    for (int i = 0; i < 10; ++i) Lsh[10 * t + i] = Li[i];
#pragma unroll
    for (int a = 0; a < 4; ++a) wsh[4 * t + a] = w[a];
  } else {
    span = 0;
    jhi = -1;
  }
  pinf[t] = make_int4(pi.y >> 8, span, pm.x, jhi);
  pob[t] = make_int2(pm.z, pm.w);
  for (int k = 0; k < span; ++k) cmap[pm.w + k] = (uint8_t)t;
  return fail;
}

// Cell waves: thread per cell (point p, block b) of batch B.  E_{p,b} = sum_o G_o J~c,o with
// G_o = L^-1 J~p,o^T (4 x 2), written straight into the point's operand tiles: window column c = 6 b + a - c0w
// goes to tile c >> 4, lane (c & 15) + 16 k.  A point observed once in every block of its span (obs sorted by
// block at load) finds its observation at a fixed offset; others read the cell records.  The first and last
// cell of a point also zero the columns of its tiles 0 .. jhi outside its span.
// Each thread takes two cells per round and issues the loads of both (the common single-observation cells:
// J pairs and scales) before either's arithmetic, so two cells' memory latencies overlap (the same
// arithmetic in the same order as one cell at a time: the same bits).
struct CellOps {
  double2 jp[4], jc[6];
  double4 s4;
  double sc[6];
};
__device__ __forceinline__ void cell_load(const Dev& d, const double* J, int o, int b, int p, CellOps& c) {
#pragma unroll
  for (int i = 0; i < 4; ++i) c.jp[i] = jload2(J, o, 7 + i);   // (pairs 0-6: r, Jc)
#pragma unroll
  for (int i = 0; i < 6; ++i) c.jc[i] = jload2(J, o, 1 + i);   // (pair 0: r)
  c.s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
#pragma unroll
  for (int i = 0; i < 6; ++i) c.sc[i] = d.scale_c[6 * b + i];
}
// E_{p,b} += (or =) the observation's G J~c from preloaded operands (load_Jp_scaled / load_Jc_scaled's
// arithmetic)
template <typename At>
__device__ __forceinline__ void cell_apply(const CellOps& c, const double* L, int col0, bool first, At at) {
  double G[4][2];
  {
    const double sp[4] = {c.s4.x, c.s4.y, c.s4.z, c.s4.w};
    double Jp[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      Jp[2 * i] = c.jp[i].x * sp[(2 * i) % 4];
      Jp[2 * i + 1] = c.jp[i].y * sp[(2 * i + 1) % 4];
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      double g0 = 0.0, g1 = 0.0;
#pragma unroll
      for (int m = 0; m <= kk; ++m) {
        g0 += L[l4(kk, m)] * Jp[m];
        g1 += L[l4(kk, m)] * Jp[4 + m];
      }
      G[kk][0] = g0;
      G[kk][1] = g1;
    }
  }
  double Jc[12];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    Jc[2 * i] = c.jc[i].x * c.sc[(2 * i) % 6];
    Jc[2 * i + 1] = c.jc[i].y * c.sc[(2 * i + 1) % 6];
  }
  if (first) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int a = 0; a < 6; ++a) at(col0 + a, kk) = G[kk][0] * Jc[a] + G[kk][1] * Jc[6 + a];
  } else {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int a = 0; a < 6; ++a) at(col0 + a, kk) += G[kk][0] * Jc[a] + G[kk][1] * Jc[6 + a];
  }
}
__device__ __forceinline__ void schur_cells(const Dev& d, const double* J, const SchurBatch& B, int tid, int c0w,
                                            const double* Lsh,
                                            const int4* pinf, const int2* pob, const uint8_t* cmap, double* Xb) {
  const int ncell = B.c1 - B.c0;
  constexpr int kStride = 64 * kSchurCellWaves;
  // cells per thread and round: 2 with four MFMA waves (their loads overlap); 1 with eight, whose register budget
  // (three waves per SIMD) does not hold two cells' operands
  constexpr int kCpt = kSchurCWaves > 4 ? 1 : 2;
  for (int lc0 = tid; lc0 < ncell; lc0 += kCpt * kStride) {
    // both cells' table entries and, for single-observation cells, their operand loads first
    int tc[kCpt], bc[kCpt], oc[kCpt];
    bool simple[kCpt];
    CellOps ops[kCpt];
#pragma unroll
    for (int h = 0; h < kCpt; ++h) {
      const int lc = lc0 + h * kStride;
      simple[h] = false;
      oc[h] = -1;
      tc[h] = 0;
      bc[h] = 0;
      if (lc < ncell) {
        const int t = cmap[lc];
        const int4 pi = pinf[t];
        const int2 po = pob[t];
        tc[h] = t;
        bc[h] = pi.x + (lc - po.y);
        if (po.x >= 0) {
          simple[h] = true;
          oc[h] = po.x + (bc[h] - pi.x);
          cell_load(d, J, oc[h], bc[h], B.p0 + t, ops[h]);
        }
      }
    }
#pragma unroll
    for (int h = 0; h < kCpt; ++h) {
      const int lc = lc0 + h * kStride;
      if (lc >= ncell) break;
      const int t = tc[h];
      const int4 pi = pinf[t];
      const int b = bc[h];
      const double* L = Lsh + 10 * t;
      double* xp = Xb + pi.z;
      const int col0 = 6 * b - c0w;
      auto at = [&](int col, int k) -> double& { return xp[64 * (col >> 4) + 16 * k + (col & 15)]; };
      if (b == pi.x)   // left margin: the columns of tiles 0 .. jhi before the span (the consumer reads them all)
        for (int col = 0; col < col0; ++col)
#pragma unroll
          for (int k = 0; k < 4; ++k) at(col, k) = 0.0;
      if (b == pi.x + pi.y - 1)   // right margin: after the span, to the end of tile jhi
        for (int col = col0 + 6; col < 16 * (pi.w + 1); ++col)
#pragma unroll
          for (int k = 0; k < 4; ++k) at(col, k) = 0.0;
      if (simple[h]) {
        cell_apply(ops[h], L, col0, true, at);
        continue;
      }
      const int4 ci = d.cells[B.c0 + lc];   // first observation (-1: none), point, (block << 16) | further, offset
      const int o0 = ci.x;
      const int k1 = ci.w;
      const int k2 = ci.w + (ci.z & 0xffff);
      if (o0 < 0) {
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
          for (int k = 0; k < 4; ++k) at(col0 + a, k) = 0.0;
        continue;
      }
#pragma unroll 1
      for (int k = k1 - 1; k < k2; ++k) {
        const int o = k < k1 ? o0 : d.cell_obs[k];
        CellOps c;
        cell_load(d, J, o, b, B.p0 + t, c);
        cell_apply(c, L, col0, k < k1, at);
      }
    }
  }
}

// Diagnostic stamps (SG_STAMP=1): workgroup 0, lane 0 of the first cell wave (slots 32-36), the point wave
// (35, 37) and the first MFMA wave (40-45) accumulate s_memtime deltas per phase.
#define SG_SSTAMP(slot)                                                                  \
  if (d.stamps && seg == 0 && lane == 0 && (wave == 0 || wave == kSchurCellWaves || wave == kSchurCellWaves + 1)) { \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                       \
    d.stamps[(slot)] += now_ - last_;                                                    \
    last_ = now_;                                                                        \
  }
// fin (one rank, after a solve's first iteration): workgroup 0 runs k_cam_finalize's pass (mode 0, taking an
// accepted step's candidate blocks) beside the segments — independent work (the segments read the decision's
// radius and slot, taken by the previous launch; the pass writes what k_S_reduce reads), one launch less.
__global__ __launch_bounds__(kSchurThreads) void k_schur(Dev d, int fin) {
  const LmState* st = d.st;
  __shared__ SchurLds sh;
  if (fin && blockIdx.x == 0) {
    cam_finalize_body(d, 0, 2, FinLds::carve(&sh.X[0][0]));
    return;
  }
  const int seg = (int)blockIdx.x - fin;
  if (seg >= d.nseg) return;
  unsigned long long last_ = __builtin_amdgcn_s_memtime();
  // the segment's descriptor load goes out beside LmState's (see k_S_reduce)
  const SchurSeg sg = d.segs[seg];
  if (st->done) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nbt = sg.bt1 - sg.bt0;
  const int c0w = 16 * sg.t0;
  double* slab = d.S_slab + sg.s_off;
  double linfail = 0.0;
  if (wave < kSchurCellWaves) {
    SG_SSTAMP(32)
    __syncthreads();
    SG_SSTAMP(33)
    for (int s = 0; s <= nbt; ++s) {
      if (s < nbt)
        schur_cells(d, d.J[st->cur], d.sbatch[sg.bt0 + s], tid, c0w, sh.L[s % 3], sh.pinf[s % 3], sh.pob[s % 3], sh.cmap[s % 3],
                    sh.X[s & 1]);
      SG_SSTAMP(34)
      __syncthreads();
      SG_SSTAMP(36)
    }
  } else if (wave == kSchurCellWaves) {
    // the point wave
    if (nbt > 0) linfail += schur_points(d, st, d.sbatch[sg.bt0], lane, sh.L[0], sh.w[0], sh.pinf[0], sh.pob[0], sh.cmap[0]);
    __syncthreads();
    for (int s = 0; s <= nbt; ++s) {
      if (s + 1 < nbt) {
        const int q = (s + 1) % 3;
        linfail += schur_points(d, st, d.sbatch[sg.bt0 + s + 1], lane, sh.L[q], sh.w[q], sh.pinf[q], sh.pob[q],
                                sh.cmap[q]);
      }
      SG_SSTAMP(35)
      __syncthreads();
      SG_SSTAMP(37)
    }
  } else {
    // MFMA waves: wave cw owns the augmented window slots u = cw + kSchurCWaves s
    const int cw = wave - kSchurCellWaves - 1;
    f64x4 acc[kSchurTPW];
#pragma unroll
    for (int s = 0; s < kSchurTPW; ++s) acc[s] = f64x4{0.0, 0.0, 0.0, 0.0};
    SG_SSTAMP(40)
    __syncthreads();
    SG_SSTAMP(41)
    for (int s = 0; s <= nbt; ++s) {
      if (s >= 1) {
        const SchurBatch B = d.sbatch[sg.bt0 + s - 1];
        const int npts = B.p1 - B.p0;
        const double* Xb = sh.X[(s - 1) & 1];
        const double* wsh = sh.w[(s - 1) % 3];
        const int4* pinf = sh.pinf[(s - 1) % 3];
        switch (cw) {
#define SG_SCHUR_CASE(W) \
          case W: schur_wave_batch<W>(acc, Xb, wsh, pinf, npts, lane); break;
          SG_SCHUR_CASE(0) SG_SCHUR_CASE(1) SG_SCHUR_CASE(2) SG_SCHUR_CASE(3)
#if SG_SCHUR_CW > 4
          SG_SCHUR_CASE(4) SG_SCHUR_CASE(5) SG_SCHUR_CASE(6) SG_SCHUR_CASE(7)
#endif
#undef SG_SCHUR_CASE
        }
        SG_SSTAMP(42)
      }
      __syncthreads();
      SG_SSTAMP(44)
    }
    mfma_drain();
    switch (cw) {
#define SG_SCHUR_CASE(W) \
      case W: schur_store<W>(acc, slab, sg.ntw, lane); break;
      SG_SCHUR_CASE(0) SG_SCHUR_CASE(1) SG_SCHUR_CASE(2) SG_SCHUR_CASE(3)
#if SG_SCHUR_CW > 4
      SG_SCHUR_CASE(4) SG_SCHUR_CASE(5) SG_SCHUR_CASE(6) SG_SCHUR_CASE(7)
#endif
#undef SG_SCHUR_CASE
    }
    SG_SSTAMP(45)
  }
  linfail = block_sum<kSchurThreads>(linfail, sh.red);
  if (tid == 0) d.seg_fail[seg] = linfail;
}

// A point spanning more blocks than a segment window (a whole-map solve's long track): one workgroup, the
// observation pairs (s <= t) of the point, each 6x6 block -A_c,s^T (P_s A_p,t^T) A_c,t into S_wide and the
// rhs terms into rhs with global atomics (k_S_reduce adds both).
__device__ __forceinline__ void schur_pair_add(double* dst, int ld, const double* Jcs, const double* Ps,
                                               const double* Jpt, const double* Jct, bool same_obs,
                                               bool same_blk, bool s_first) {
  double M[2][2];
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)
#pragma unroll
    for (int u = 0; u < 2; ++u)
      M[rr][u] = Ps[4 * rr] * Jpt[4 * u] + Ps[4 * rr + 1] * Jpt[4 * u + 1] + Ps[4 * rr + 2] * Jpt[4 * u + 2] +
                 Ps[4 * rr + 3] * Jpt[4 * u + 3];
  double N[6][2];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int u = 0; u < 2; ++u) N[a][u] = Jcs[a] * M[0][u] + Jcs[6 + a] * M[1][u];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const double Tac = N[a][0] * Jct[c] + N[a][1] * Jct[6 + c];
      const double Tca = N[c][0] * Jct[a] + N[c][1] * Jct[6 + a];
      double v;
      if (same_obs) v = Tac;
      else if (same_blk) v = Tac + Tca;
      else if (s_first) v = Tac;
      else v = Tca;
      atomicAdd(dst + a * ld + c, -v);
    }
}

__global__ __launch_bounds__(kSchurThreads) void k_schur_wide(Dev d) {
  const LmState* st = d.st;
  if (st->done || (int)blockIdx.x >= d.nwide) return;
  __shared__ double vinv[10], tpv[4];
  const WideSeg ws = d.wsegs[blockIdx.x];
  const int p = ws.p, tid = threadIdx.x;
  if (!d.pfree[p]) return;
  if (tid == 0) {
    double Vi[10], Li[10], w[4];
    d.seg_fail[d.nseg + blockIdx.x] = point_block(d, st, p, Vi, Li, w) ? 0.0 : 1.0;
#pragma unroll
    for (int i = 0; i < 10; ++i) vinv[i] = Vi[i];
#pragma unroll
    for (int a = 0; a < 4; ++a) tpv[a] = d.tp[4 * (size_t)p + a];
  }
  __syncthreads();
  const int obs_lo = d.poff[p], obs_hi = d.poff[p + 1];
  const double4 s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
  const double* Jw = d.J[st->cur];
  for (int o = obs_lo + tid; o < obs_hi; o += kSchurThreads) {
    const int b = d.frame_block[d.obs_frame[o]];
    if (b < 0) continue;
    double Jp[8], Jc[12];
    load_Jp_scaled(Jw, o, s4, Jp);
    load_Jc_scaled(d, Jw, o, b, Jc);
    const double e0 = Jp[0] * tpv[0] + Jp[1] * tpv[1] + Jp[2] * tpv[2] + Jp[3] * tpv[3];
    const double e1 = Jp[4] * tpv[0] + Jp[5] * tpv[1] + Jp[6] * tpv[2] + Jp[7] * tpv[3];
#pragma unroll
    for (int a = 0; a < 6; ++a) atomicAdd(d.rhs + 6 * b + a, -(Jc[a] * e0 + Jc[6 + a] * e1));
  }
  for (int k = ws.pair_lo + tid; k < ws.pair_hi; k += kSchurThreads) {
    const int2 pr = d.pairs[k];
    const int os = obs_lo + (pr.x >> 16), ot = obs_lo + (pr.x & 0xffff);
    const int bs = pr.y >> 16, bt = pr.y & 0xffff;
    double Jcs[12], Jct[12], Jpt[8], Jps[8], Ps[8];
    load_Jc_scaled(d, Jw, os, bs, Jcs);
    load_Jc_scaled(d, Jw, ot, bt, Jct);
    load_Jp_scaled(Jw, ot, s4, Jpt);
    load_Jp_scaled(Jw, os, s4, Jps);
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        double a = 0.0;
#pragma unroll
        for (int m = 0; m < 4; ++m) a += Jps[4 * rr + m] * sym4(vinv, m, c);
        Ps[4 * rr + c] = a;
      }
    const int I = bs < bt ? bs : bt, Jb = bs < bt ? bt : bs;
    schur_pair_add(d.S_wide + (size_t)(6 * I) * d.n + 6 * Jb, d.n, Jcs, Ps, Jpt, Jct, os == ot, bs == bt, bs < bt);
  }
}

// ------------------------------------------------------------------------------------------------
// The camera-camera terms of the damped reduced system that do not come from the Schur complement:
// blockdiag(U) (observation Jacobians) + FrameDistance diagonal and cross blocks + D^2 = diag/radius,
// all Jacobi-scaled, for element (6I+a, 6J+c), J >= I.
//
// k_S_reduce: one workgroup per 16x16 tile (R <= C) of the band of S (the frame columns), then one per rhs
// block.  A tile's partials (one per segment whose window covers it, in segment order) are split over the four
// waves (partial k to wave k mod 4, every lane summing 4 elements, 8 partials in flight), the four wave sums
// combined in wave order (deterministic); then each thread finishes one element: the wide-point accumulator
// and, on the assembling rank, the camera-only terms.  S leaves here damped; elements below the diagonal of a
// diagonal tile are written as 0 (no factorisation reads them).  Tiles outside the band are never written
// (zero since the load).
// amode: 0 this rank adds no camera-only terms (landmark shards: ranks > 0 in a solve's first iteration);
// 1 blockdiag(U) of the summed camera blocks + FrameDistance + damping (one rank; rank 0 of shards in the
// first iteration); 2 this rank's own camera blocks, the FrameDistance terms on rank 0, no damping (landmark
// shards after the first iteration: summed with S in one exchange, k_cam_finalize mode 2 adds the damping).
__global__ __launch_bounds__(256) void k_S_reduce(Dev d, int amode) {
  // LmState is read beside the first work-list loads, not ahead of them: the done test comes after the
  // partial walk (a finished solve's trailing launches walk once more; every other launch saves a round trip)
  const LmState* st = d.st;
  const int done = st->done;
  const double radius = st->radius;
  const int tid = threadIdx.x, lane = tid & 63, part = tid >> 6;
  const int wv = blockIdx.x;
  if (wv >= d.nstile + d.NB) return;
  const int nf = 6 * d.NB;   // frame columns
  if (wv < d.nstile) {
    const int rc = d.stile[wv];
    const int R = rc >> 16, C = rc & 0xffff;
    const int i = 16 * R + (tid >> 4), j = 16 * C + (tid & 15);
    const bool live = i < nf && j < nf;
    const bool up = live && i <= j;
    const size_t gi = (size_t)(live ? i : 0) * d.n + (live ? j : 0);
    // epilogue operands first, so their round trips overlap the partial walk
    const double e_acc = (up && d.nwide) ? d.S_wide[gi] : 0.0;
    const int I = i / 6, a = i - 6 * (i / 6), Jb = j / 6, c = j - 6 * (j / 6);
    double e_si = 0.0, e_sj = 0.0, e_u = 0.0, e_fd = 0.0, e_dg = 0.0, e_x = 0.0;
    const bool fd_here = amode == 1 || (amode == 2 && d.rank == 0);
    if (amode != 0 && up) {
      e_si = d.scale_c[i];
      e_sj = d.scale_c[j];
      if (I == Jb) {
        e_u = (amode == 2 ? d.xcam_loc : d.xchg_cam)[(size_t)I * kCamV + u6(a, c)];
        e_fd = (fd_here && a >= 3 && c >= 3) ? d.fd_D[9 * I + 3 * (a - 3) + (c - 3)] : 0.0;
        e_dg = (amode == 1 && a == c) ? d.diag_c[i] : 0.0;
      } else if (fd_here && a >= 3 && c >= 3) {
        const int dd = d.fd_pair[I * d.NB + Jb];
        if (dd >= 0) {
          const double* Xd = d.fd_X + 9 * dd;   // J_a J_b^T, rows: frame a's translation
          e_x = d.frame_block[d.fd_a[dd]] == I ? Xd[3 * (a - 3) + (c - 3)] : Xd[3 * (c - 3) + (a - 3)];
        }
      }
    }
    const int j0 = d.s_loff[wv], j1 = d.s_loff[wv + 1];
    __shared__ double wsum[4][256];
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    constexpr int kSR = 8;
    for (int base = j0 + part; base < j1; base += 4 * 64) {
      const int cnt = min(64, (j1 - base + 3) / 4);
      const int myoff = d.s_lidx[lane < cnt ? base + 4 * lane : j0];
      for (int k = 0; k < cnt; k += kSR) {
        double v[kSR][4];
#pragma unroll
        for (int u = 0; u < kSR; ++u) {
          const double* src = d.S_slab + __builtin_amdgcn_readlane(myoff, min(k + u, 63)) + lane;
#pragma unroll
          for (int m = 0; m < 4; ++m) v[u][m] = src[64 * m];
        }
#pragma unroll
        for (int u = 0; u < kSR; ++u)
          if (k + u < cnt)
#pragma unroll
            for (int m = 0; m < 4; ++m) s[m] += v[u][m];
      }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) wsum[part][lane + 64 * m] = s[m];
    __syncthreads();
    if (done || !live) return;
    if (!up) {
      d.S[gi] = 0.0;
      if (d.nwide) d.S_wide[gi] = 0.0;   // schur_pair_add also adds a diagonal block's lower half: keep it clean
      return;
    }
    double t = ((wsum[0][tid] + wsum[1][tid]) + wsum[2][tid]) + wsum[3][tid];
    t += e_acc;
    if (d.nwide) d.S_wide[gi] = 0.0;
    if (amode != 0) {   // assembly_term, from the prefetched operands
      double v;
      if (I == Jb) {
        v = (e_u + e_fd) * (e_si * e_sj);
        if (a == c) v += e_dg / radius;
      } else {
        v = e_x * e_si * e_sj;
      }
      t += v;
    }
    d.S[gi] = t;
    return;
  }
  // rhs block I: one wave per 64-entry chunk of its partial list (in list order), lanes 0..5
  const int I = wv - d.nstile;
  // speculative linearization: clear block I of the candidate slot's wide-chunk camera accumulator before
  // k_update_lin adds to it (k_cam_reduce keeps the current slot's)
  if (d.spec && part == 1 && lane < kCamV) d.cam_wide[st->cur ^ 1][(size_t)I * kCamV + lane] = 0.0;
  const int j0 = d.r_loff[I], j1 = d.r_loff[I + 1];
  const int el = lane < 6 ? lane : 0;
  const int ei = 6 * I + el;
  const double e_acc = d.rhs[ei];
  const double e_si = amode != 0 ? d.scale_c[ei] : 0.0, e_g = amode != 0 ? d.camg[ei] : 0.0;
  __shared__ double rsum[4][6];
  constexpr int kSR = 32;
  double s = 0.0;
  int myoff = d.r_lidx[(j0 + 64 * part + lane < j1) ? j0 + 64 * part + lane : 0];
  for (int base = j0 + 64 * part; base < j1; base += 256) {
    const int cnt = min(64, j1 - base);
    const int nxt = d.r_lidx[(base + 256 + lane < j1) ? base + 256 + lane : 0];
    for (int k = 0; k < cnt; k += kSR) {
      double v[kSR];
#pragma unroll
      for (int u = 0; u < kSR; ++u) v[u] = d.S_slab[__builtin_amdgcn_readlane(myoff, min(k + u, 63)) + el];
#pragma unroll
      for (int u = 0; u < kSR; ++u)
        if (k + u < cnt) s += v[u];
    }
    myoff = nxt;
  }
  if (lane < 6) rsum[part][lane] = s;
  __syncthreads();
  if (done || part != 0 || lane >= 6) return;
  s = ((rsum[0][lane] + rsum[1][lane]) + rsum[2][lane]) + rsum[3][lane];
  s += e_acc;
  if (amode != 0) s += e_si * e_g;   // y = rhs_sub + S g_c
  d.xc[ei] = s;       // local rhs partial (all-reduced with S); the wide accumulator is reset
  d.rhs[ei] = 0.0;
}

// ------------------------------------------------------------------------------------------------
// Landmark shards: the part of S the Cholesky reads (per 16-row panel, columns kb .. band end, row-major)
// and the rhs, packed into one contiguous buffer for the all-reduce and unpacked after it.  Outside the
// band every rank's S holds exact zeros (k_S_reduce writes every block pair), so only the band travels.
// Block (pk, y) of the grid copies panel pk (pk == npanel: the rhs).
__global__ __launch_bounds__(256) void k_S_pack(double* S, int n, const int32_t* panel_jend, const int32_t* off,
                                                int npanel, double* buf, int unpack) {
  const int pk = blockIdx.x;
  const int stride = 256 * gridDim.y;
  if (pk == npanel) {
    double* xc = S + (size_t)n * n;
    for (int i = blockIdx.y * 256 + threadIdx.x; i < n; i += stride) {
      if (unpack) xc[i] = buf[off[npanel] + i];
      else buf[off[npanel] + i] = xc[i];
    }
    return;
  }
  const int kb = pk * kCholNb, w = min(kCholNb, n - kb), width = panel_jend[pk] - kb;
  const int cnt = w * width;
  for (int e = blockIdx.y * 256 + threadIdx.x; e < cnt; e += stride) {
    const int r = e / width, c = e - r * width;
    const size_t gi = (size_t)(kb + r) * n + kb + c;
    if (unpack) S[gi] = buf[off[pk] + e];
    else buf[off[pk] + e] = S[gi];
  }
}

// ------------------------------------------------------------------------------------------------
// Free intrinsics (SolveAllFrames(..., solve_cameras = true), slam.cpp:447-480; the oracle's k_col_ layout).
// Each camera's 7 intrinsics are 7 more columns of the reduced system, after the 6 NB frame columns:
// S = [[S_ff, S_fk], [., S_kk]], still eliminated over the points.  Few columns, coupled to every frame
// and point of the camera, so these kernels are plain thread-per-item passes with global atomics (not on
// the SolveFrames hot path); the k columns make S dense, so the Cholesky runs its global-memory variant.
//   k_intr_zero / k_intr_lin / k_intr_fin (after an accepted step): J_k per observation, the k columns
//     of J^T J (KU), the k gradient and diagonal, CameraStabilization (slam.cpp:107-124) on camera c;
//   k_intr_assemble + k_intr_schur (every iteration): the k columns of the damped, scaled S and rhs:
//     KU + damping, minus sum_p W_kp V~p^-1 [W_fp W_kp]^T;
//   k_intr_step (after the solve): candidate intrinsics k+ = k - S x_k, step norms, stabilization
//     model term and candidate cost.  The observation model terms take A_k x_k in k_point_update.

constexpr int kIntrCamV = 42;   // per camera: upper 7x7 of J_k^T J_k (28), J_k^T r (7), diagonal (7)
constexpr int kIntrKMax = 7 * kMaxIntrCams;
__global__ __launch_bounds__(256) void k_intr_zero(Dev d) {
  const LmState* st = d.st;
  if (st->done || !st->need_lin) return;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < d.n * d.nk) d.KU[i] = 0.0;
  if (i < (d.NB + 1) * d.ncam * kIntrCamV) d.kpart[i] = 0.0;
  if (i < d.nk) {
    d.camg[d.kc0 + i] = 0.0;
    d.camdiag[d.kc0 + i] = 0.0;
  }
}

// One thread per observation: J_k (the same corrected projection Jacobian as k_linearize), stored for
// k_intr_fk, which forms the frame-intrinsics block KU_fk and the per-camera sums (upper 7x7 of J_k^T J_k, the
// gradient, the diagonal) per frame block from the observation lists, without atomics; k_intr_fin adds the
// per-block partials in block order.  (Per-observation LDS / global atomics on a few hundred shared addresses
// took 49 us at config 2.)
__global__ __launch_bounds__(256) void k_intr_lin(Dev d) {
  const LmState* st = d.st;
  if (st->done || !st->need_lin) return;
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= d.M) return;
  const int cur = st->cur;
  const int m = d.obs_meta[o], f = d.obs_frame[o], p = d.obs_pnt[o], cam = meta_cam(m);
  double* Jko = d.Jk + 14 * (size_t)o;
  const double4 Xv = reinterpret_cast<const double4*>(d.X[cur])[p];
  const double X[4] = {Xv.x, Xv.y, Xv.z, Xv.w};
  const double pt[2] = {d.obs_pt[2 * o], d.obs_pt[2 * o + 1]};
  double rr[2], Jc[12], Jp[8], Jk[14], c;
  const bool ok = !(m & kMetaFixed) && LinearizeObservation(d.q[cur] + 4 * f, d.t[cur] + 3 * f, d.k[cur] + 7 * cam,
                                                            X, pt, d.b, d.inv_b, rr, Jc, Jp, &c, Jk);
  // a failed projection fails the linearization (k_linearize) and contributes nothing
#pragma unroll
  for (int i = 0; i < 14; ++i) Jko[i] = ok ? Jk[i] : 0.0;
}

// Sum of kV values over the workgroup's waves (wave sums, then the waves in order): the result for value e is in
// red[0][e] after the call.
template <int kWaves, int kV>
__device__ __forceinline__ void wg_sum_values(const double (&v)[kV], double (*red)[kV]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < kV; ++e) {
    const double t = wave_sum_full(v[e]);   // DPP (every lane active here)
    if (lane == 0) red[wave][e] = t;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kV; e += 64 * kWaves) {
    double t = red[0][e];
    for (int w = 1; w < kWaves; ++w) t += red[w][e];
    red[0][e] = t;
  }
  __syncthreads();
}

// Per frame block b (blockIdx.x; b = NB: the observations of fixed frames) and camera c (blockIdx.y), over the
// block's observation list:
//   kMode 0 (after k_intr_lin): KU_fk rows of b, columns of c: sum J_c^T J_k over the block's observations of
//     camera c (stored: one writer per entry), and the camera sums of those observations into kpart[b][c];
//   kMode 1 (after k_intr_schur): S_fk rows of b, columns of c -= sum over the block's observations of free
//     points of A_c^T (A_p Y_pc^T) (Y_pc = W_kp V~p^-1 of camera c, k_intr_schur).
#ifndef SG_INTR_FK_THREADS
#define SG_INTR_FK_THREADS 256
#endif
constexpr int kIntrFkThreads = SG_INTR_FK_THREADS;   // (the slices per block list stay ~256 observations)
template <int kMode>
__global__ __launch_bounds__(kIntrFkThreads) void k_intr_fk(Dev d, int nsl) {
  const LmState* st = d.st;
  if (st->done) return;
  if (kMode == 0 && !st->need_lin) return;
  constexpr int kV = kMode == 0 ? 2 * kIntrCamV : kIntrCamV;
  constexpr int kW = kIntrFkThreads / 64;
  __shared__ double red[kW][kV];
  // workgroup (b, slice sl) of blockIdx.x takes the sl-th part of block b's list
  // SG_STAMP=1: one mid-grid workgroup's thread 0 times its steps (d.stamps[58 + 3 kMode ..]; 48-56: k_chol_border)
  const bool stw = d.stamps && blockIdx.x == gridDim.x / 2 && blockIdx.y == 0 && threadIdx.x == 0;
  unsigned long long t0s = 0;
  auto nowt = []() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
    return t;
  };
  if (stw) t0s = nowt();
  const int b = blockIdx.x / nsl, sl = blockIdx.x - b * nsl, c = blockIdx.y, tid = threadIdx.x, cur = st->cur;
  const int nk = d.nk, ncam = d.ncam;
  const int l0 = d.intr_boff[b], len = d.intr_boff[b + 1] - l0;
  const int i0 = l0 + (int)((long long)len * sl / nsl), i1 = l0 + (int)((long long)len * (sl + 1) / nsl);
  double acc[kV];
#pragma unroll
  for (int e = 0; e < kV; ++e) acc[e] = 0.0;
  const double* J = d.J[cur];
  for (int i = i0 + tid; i < i1; i += kIntrFkThreads) {
    const int o = d.intr_bidx[i];
    const int m = d.obs_meta[o];
    if constexpr (kMode == 0) {
      if (meta_cam(m) != c) continue;
      const double* Jko = d.Jk + 14 * (size_t)o;
      double Jk[14], r[2], Jc[12];
#pragma unroll
      for (int e = 0; e < 14; ++e) Jk[e] = Jko[e];
      const double2 rv = jload2(J, o, 0);
      r[0] = rv.x;
      r[1] = rv.y;
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        const double2 v = jload2(J, o, 1 + e);   // raw J_c (zero outside the frame's free parts)
        Jc[2 * e] = v.x;
        Jc[2 * e + 1] = v.y;
      }
      if (b < d.NB) {
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
          for (int j = 0; j < 7; ++j) acc[7 * a + j] += Jc[a] * Jk[j] + Jc[6 + a] * Jk[7 + j];
      }
      double* ka = acc + kIntrCamV;
      int u = 0;
#pragma unroll
      for (int a = 0; a < 7; ++a) {
#pragma unroll
        for (int j = a; j < 7; ++j) ka[u++] += Jk[a] * Jk[j] + Jk[7 + a] * Jk[7 + j];
        ka[28 + a] += Jk[a] * r[0] + Jk[7 + a] * r[1];
        ka[35 + a] += Jk[a] * Jk[a] + Jk[7 + a] * Jk[7 + a];
      }
    } else {
      if (!(m & kMetaPfree)) continue;
      const int p = d.obs_pnt[o];
      const double4 s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
      const double sp[4] = {s4.x, s4.y, s4.z, s4.w};
      double r[2], Jc[12], Jp[8];
      load_scaled_J(d, J, o, b, sp, r, Jc, Jp);
      const double* Y = d.Yk + ((size_t)p * ncam + c) * 28;
      double Mx[14];   // A_p Y^T (2x7)
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int j = 0; j < 7; ++j) {
          double v = 0.0;
#pragma unroll
          for (int a = 0; a < 4; ++a) v += Jp[4 * rr + a] * Y[4 * j + a];
          Mx[7 * rr + j] = v;
        }
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int j = 0; j < 7; ++j) acc[7 * a + j] -= Jc[a] * Mx[j] + Jc[6 + a] * Mx[7 + j];
    }
  }
  unsigned long long t1s = 0, t2s = 0;
  if (stw) t1s = nowt();
  wg_sum_values<kW, kV>(acc, red);
  if (stw) t2s = nowt();
  // the slices of a block add into KU_fk / S_fk (nsl atomics per entry); the camera sums go to their partial slot
  if constexpr (kMode == 0) {
    for (int e = tid; e < kV; e += kIntrFkThreads) {
      if (e < kIntrCamV) {
        if (b < d.NB) atomicAdd(d.KU + (size_t)(6 * b + e / 7) * nk + 7 * c + e % 7, red[0][e]);
      } else {
        atomicAdd(d.kpart + ((size_t)b * ncam + c) * kIntrCamV + e - kIntrCamV, red[0][e]);   // (nsl slices)
      }
    }
  } else {
    for (int e = tid; e < kV; e += kIntrFkThreads)
      atomicAdd(d.S + (size_t)(6 * b + e / 7) * d.n + d.kc0 + 7 * c + e % 7, red[0][e]);
  }
  if (stw) {
    const unsigned long long t3s = nowt();
    d.stamps[58 + 3 * kMode] += t1s - t0s;
    d.stamps[59 + 3 * kMode] += t2s - t1s;
    d.stamps[60 + 3 * kMode] += t3s - t2s;
  }
}

__device__ __forceinline__ void stab_residual(const double* k, double* res, double* J) {
  res[0] = 1000.0 * k[0] * k[0];
  res[1] = 1000.0 * k[1] * k[1];
  res[2] = 1000.0 * k[2] * k[2];
  res[3] = 0.1 * (k[3] - 416.0) * (k[3] - 416.0);
  res[4] = 0.1 * (k[4] + k[3]) * (k[4] + k[3]);
  res[5] = 0.01 * (k[5] - 320.0) * (k[5] - 320.0);
  res[6] = 0.01 * (k[6] - 240.0) * (k[6] - 240.0);
  if (!J) return;
  for (int i = 0; i < 49; ++i) J[i] = 0.0;
  J[0] = 2000.0 * k[0];
  J[8] = 2000.0 * k[1];
  J[16] = 2000.0 * k[2];
  J[24] = 0.2 * (k[3] - 416.0);
  J[31] = J[32] = 0.2 * (k[4] + k[3]);
  J[40] = 0.02 * (k[5] - 320.0);
  J[48] = 0.02 * (k[6] - 240.0);
}

// One wave: stabilization terms of every camera (lane = camera), then the cost, |g|_inf of the k columns
// and |k|^2 into the exchange slots k_cam_finalize reads.
constexpr int kIntrFinThreads = 256;
__global__ __launch_bounds__(kIntrFinThreads) void k_intr_fin(Dev d, int nsl) {
  LmState* st = d.st;
  if (st->done || !st->need_lin) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, cur = st->cur, nk = d.nk;
  // the per-block camera sums of k_intr_fk<0> (NB + 1 partials per value): h threads per value, each summing
  // every h-th block, then the h parts in order
  __shared__ double part[kIntrFinThreads];
  const int nv = d.ncam * kIntrCamV, h = max(1, kIntrFinThreads / nv), np = d.NB + 1;
  {
    const int v = tid / h, hh = tid - v * h;
    double t = 0.0;
    if (v < nv) {
      const int cam = v / kIntrCamV, e = v - cam * kIntrCamV;
      for (int q0 = hh; q0 < np; q0 += 8 * h) {
        double u[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int q = q0 + k * h;
          u[k] = q < np ? d.kpart[((size_t)q * d.ncam + cam) * kIntrCamV + e] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) t += u[k];
      }
    }
    part[tid] = t;
  }
  __syncthreads();
  for (int v = tid; v < nv; v += kIntrFinThreads) {
    const int cam = v / kIntrCamV, e = v - cam * kIntrCamV, kc = 7 * cam;
    double t = 0.0;
    for (int hh = 0; hh < h; ++hh) t += part[v * h + hh];
    if (e < 28) {
      int a = 0, u = e;
      while (u >= 7 - a) {
        u -= 7 - a;
        ++a;
      }
      d.KU[(size_t)(d.kc0 + kc + a) * nk + kc + a + u] += t;
    } else if (e < 35) {
      d.camg[d.kc0 + kc + (e - 28)] += t;
    } else {
      d.camdiag[d.kc0 + kc + (e - 35)] += t;
    }
  }
  __syncthreads();
  double cost = 0.0, xn2 = 0.0;
  if (tid < d.ncam) {   // (wave 0 from here)
    const double* k = d.k[cur] + 7 * lane;
    double res[7], J[49];
    stab_residual(k, res, J);
    double sq = 0.0;
    for (int i = 0; i < 7; ++i) sq += res[i] * res[i];
    double rho0, rho1;
    Cauchy(sq, d.stab_b, d.stab_inv_b, &rho0, &rho1);
    cost = 0.5 * rho0;
    const double sr = sqrt(rho1);
    // the corrected residual and Jacobian in registers (k_intr_step reads the stored copy)
    double kr[7], kj[49];
#pragma unroll
    for (int i = 0; i < 7; ++i) kr[i] = sr * res[i];
#pragma unroll
    for (int i = 0; i < 49; ++i) kj[i] = sr * J[i];
    double* ks = d.kst + 56 * lane;
#pragma unroll
    for (int i = 0; i < 7; ++i) ks[i] = kr[i];
#pragma unroll
    for (int i = 0; i < 49; ++i) ks[7 + i] = kj[i];
    const int kc = 7 * lane;
    double* Kk = d.KU + (size_t)(d.kc0 + kc) * nk;
#pragma unroll
    for (int a = 0; a < 7; ++a) {
      double g = 0.0, dg = 0.0;
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        g += kj[7 * i + a] * kr[i];
        dg += kj[7 * i + a] * kj[7 * i + a];
      }
      d.camg[d.kc0 + kc + a] += g;
      d.camdiag[d.kc0 + kc + a] += dg;
#pragma unroll
      for (int j = a; j < 7; ++j) {
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < 7; ++i) v += kj[7 * i + a] * kj[7 * i + j];
        Kk[(size_t)a * nk + kc + j] += v;
      }
    }
    for (int i = 0; i < 7; ++i) xn2 += k[i] * k[i];
  }
  __syncthreads();
  if (wave != 0) return;
  double gm = 0.0;
  for (int i = lane; i < nk; i += 64) gm = fmax(gm, fabs(d.camg[d.kc0 + i]));
  gm = wave_max(gm);
  cost = wave_sum_full(cost);
  xn2 = wave_sum_full(xn2);
  if (lane == 0) {
    double* xs = d.xchg_cam + (size_t)d.NB * kCamV;
    xs[kXCost] += cost;
    xs[kXNum] = fmax(xs[kXNum], gm);   // single rank (Load rejects shards with free intrinsics)
    if (st->first) xs[kXXnorm2] += xn2;
  }
}

// The k columns of the damped, scaled S (upper triangle) and the k part of the rhs y = s g, before the
// point-elimination terms of k_intr_schur.  Thread per (row, k column).
__global__ __launch_bounds__(256) void k_intr_assemble(Dev d) {
  const LmState* st = d.st;
  if (st->done) return;
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= d.n * d.nk) return;
  const int i = id / d.nk, j = id - i * d.nk, col = d.kc0 + j;
  if (i <= col) {
    double v = d.KU[id] * d.scale_c[i] * d.scale_c[col];
    if (i == col) v += d.diag_c[col] / st->radius;
    d.S[(size_t)i * d.n + col] = v;
  }
  if (i == 0) d.xc[col] = d.scale_c[col] * d.camg[col];
}

// Thread per free point p: W_kp = A_k^T A_p over its observations of camera c (scaled), Y = W_kp V~p^-1, then
// S_kk -= Y W_kp'^T and rhs_k -= W_kp t_p; Y goes to Yk for the frame-intrinsics terms S_bk -= A_c^T (A_p Y^T),
// which k_intr_fk<1> sums per frame block over the block's observation list.  The k-k block of S and the k rhs
// (shared by every point) accumulate in LDS per workgroup, then one global atomic per entry and workgroup (a
// global atomic per point on ~120 shared addresses took 1.9 ms at config 2).  (The S_fk terms as LDS atomics per
// observation here took 200 us at config 2.)
struct IntrSchurLds {
  double skk[kIntrKMax * kIntrKMax], sxk[kIntrKMax];
};
__device__ __forceinline__ void intr_schur_point(const Dev& d, int p, bool act, IntrSchurLds& sh);
__global__ __launch_bounds__(128) void k_intr_schur(Dev d) {
  const LmState* st = d.st;
  if (st->done || d.P == 0) return;
  __shared__ IntrSchurLds sh;
  const int tid = threadIdx.x;
  for (int i = tid; i < kIntrKMax * kIntrKMax; i += blockDim.x) sh.skk[i] = 0.0;
  if (tid < kIntrKMax) sh.sxk[tid] = 0.0;
  __syncthreads();
  const int p = blockIdx.x * blockDim.x + tid;
  intr_schur_point(d, min(p, d.P - 1), p < d.P && d.pfree[p], sh);   // every lane: wave sums inside
  __syncthreads();
  const int K = d.nk, n = d.n;
  for (int i = tid; i < K * K; i += blockDim.x) {
    const int r = i / K, c = i - r * K;
    const double v = sh.skk[r * kIntrKMax + c];
    if (c >= r && v != 0.0) atomicAdd(d.S + (size_t)(d.kc0 + r) * n + d.kc0 + c, v);
  }
  if (tid < K && sh.sxk[tid] != 0.0) atomicAdd(d.xc + d.kc0 + tid, sh.sxk[tid]);
}

// Called by every lane (inactive ones with no observations, so W = 0): the S_kk and rhs terms, shared by all
// points, are summed over the wave first (one LDS atomic a value and wave, not 64 on one address).
__device__ __forceinline__ void intr_schur_point(const Dev& d, int p, bool act, IntrSchurLds& sh) {
  double* skk = sh.skk;
  double* sxk = sh.sxk;
  const bool lane0 = (threadIdx.x & 63) == 0;
  const int o0 = act ? d.poff[p] : 0, o1 = act ? d.poff[p + 1] : 0;
  const double4 s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
  const double sp[4] = {s4.x, s4.y, s4.z, s4.w};
  double Vi[10];
  for (int i = 0; i < 10; ++i) Vi[i] = d.Vinv[10 * (size_t)p + i];
  const double4 t4 = reinterpret_cast<const double4*>(d.tp)[p];
  const double tpv[4] = {t4.x, t4.y, t4.z, t4.w};
  // W of camera c (7x4, row-major), accumulated over the point's observations of that camera (one walk per
  // camera; loops unrolled so W, Y stay in registers)
  auto build_W = [&](int c, double (&W)[28]) -> bool {
#pragma unroll
    for (int i = 0; i < 28; ++i) W[i] = 0.0;
    bool any = false;
    for (int o = o0; o < o1; ++o) {
      const int m = d.obs_meta[o];
      if ((m & kMetaFixed) || meta_cam(m) != c) continue;
      any = true;
      const double* Jk = d.Jk + 14 * (size_t)o;
      double Jr[8];   // corrected Jp (2x4)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double2 v = jload2(d.J[d.st->cur], o, 7 + i);
        Jr[2 * i] = v.x;
        Jr[2 * i + 1] = v.y;
      }
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const double k0 = Jk[j] * d.scale_c[d.kc0 + 7 * c + j], k1 = Jk[7 + j] * d.scale_c[d.kc0 + 7 * c + j];
#pragma unroll
        for (int a = 0; a < 4; ++a) W[4 * j + a] += (k0 * Jr[a] + k1 * Jr[4 + a]) * sp[a];
      }
    }
    return any;
  };
  for (int c = 0; c < d.ncam; ++c) {
    double W[28], Y[28];
    const bool has = build_W(c, W);
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      double r = 0.0;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        double y = 0.0;
#pragma unroll
        for (int e = 0; e < 4; ++e) y += W[4 * j + e] * sym4(Vi, e, a);
        Y[4 * j + a] = has ? y : 0.0;   // (a lane without observations of c adds exact zeros)
        r += W[4 * j + a] * tpv[a];
      }
      const double rs = wave_sum_full(has ? -r : 0.0);
      if (lane0) atomicAdd(sxk + 7 * c + j, rs);
    }
    // S_kk block (c, c), upper triangle
#pragma unroll
    for (int j = 0; j < 7; ++j)
#pragma unroll
      for (int j2 = j; j2 < 7; ++j2) {
        double v = 0.0;
#pragma unroll
        for (int a = 0; a < 4; ++a) v += Y[4 * j + a] * W[4 * j2 + a];
        const double vs = wave_sum_full(-v);
        if (lane0) atomicAdd(skk + (7 * c + j) * kIntrKMax + 7 * c + j2, vs);
      }
    // blocks (c', c) of the earlier cameras: Y_c' (this lane's own store below, read back) W_c^T
    for (int c1 = 0; c1 < c; ++c1) {
      double Y1[28];
      const double* Yi = d.Yk + ((size_t)p * d.ncam + c1) * 28;
#pragma unroll
      for (int i = 0; i < 28; ++i) Y1[i] = act ? Yi[i] : 0.0;
#pragma unroll
      for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int j2 = 0; j2 < 7; ++j2) {
          double v = 0.0;
#pragma unroll
          for (int a = 0; a < 4; ++a) v += Y1[4 * j + a] * W[4 * j2 + a];
          const double vs = wave_sum_full(-v);
          if (lane0) atomicAdd(skk + (7 * c1 + j) * kIntrKMax + 7 * c + j2, vs);
        }
    }
    // Y_pc for the S_fk terms of the point's observations (k_intr_fk<1>) and the later cameras' blocks
    if (act) {
      double* Yo = d.Yk + ((size_t)p * d.ncam + c) * 28;
#pragma unroll
      for (int i = 0; i < 28; ++i) Yo[i] = Y[i];
    }
  }
}

// Candidate intrinsics k+ = k - S x_k (Euclidean, the oracle's Plus), their step / norm terms, and the
// stabilization model term and candidate cost.  Runs after the Cholesky kernel, adds to its slots.
__global__ __launch_bounds__(64) void k_intr_step(Dev d) {
  const LmState* st = d.st;
  if (st->done) return;
  const int lane = threadIdx.x, cur = st->cur, nxt = cur ^ 1;
  double step2 = 0.0, candx2 = 0.0, model = 0.0, candcost = 0.0;
  if (lane < d.ncam) {
    const double* k = d.k[cur] + 7 * lane;
    double* kn = d.k[nxt] + 7 * lane;
    const int kc = d.kc0 + 7 * lane;
    double dl[7], knv[7];
    for (int j = 0; j < 7; ++j) {
      dl[j] = -d.xc[kc + j] * d.scale_c[kc + j];
      knv[j] = k[j] + dl[j];
      kn[j] = knv[j];
      step2 += (knv[j] - k[j]) * (knv[j] - k[j]);
      candx2 += knv[j] * knv[j];
    }
    const double* ks = d.kst + 56 * lane;
    for (int i = 0; i < 7; ++i) {
      double mi = 0.0;
      for (int j = 0; j < 7; ++j) mi += ks[7 + 7 * i + j] * dl[j];
      model -= mi * (ks[i] + 0.5 * mi);
    }
    double res[7];
    stab_residual(knv, res, nullptr);
    double sq = 0.0;
    for (int i = 0; i < 7; ++i) sq += res[i] * res[i];
    double rho0, rho1;
    Cauchy(sq, d.stab_b, d.stab_inv_b, &rho0, &rho1);
    candcost = 0.5 * rho0;
  }
  step2 = wave_sum_full(step2);
  candx2 = wave_sum_full(candx2);
  model = wave_sum_full(model);
  candcost = wave_sum_full(candcost);
  if (lane == 0) {
    d.xchg_chol[kCStep2] += step2;
    d.xchg_chol[kCCandX2] += candx2;
    d.xchg_chol[kCModel] += model;
    d.xchg_chol[kCCandCost] += candcost;
  }
}

// ------------------------------------------------------------------------------------------------
// Reduced camera system solve (the SPARSE_SCHUR + CHOLMOD step behind slam.cpp:489, restated): one
// workgroup factors the damped, banded Schur complement A = U^T U (right-looking, 16-wide panels, the
// rhs carried as an augmented column), then back-substitutes.  The band (co-visibility of the sliding
// window) fits a 128x128 fp64 LDS window that slides down the diagonal; trailing updates run as
// v_mfma_f64_16x16x4 tiles.  Bands wider than the window take the global-memory path.
constexpr int kCholWS = 128;
constexpr int kPanelWaves = 3;   // 16 + 3 x 48 >= kCholWS columns
constexpr int kJendSh = 512;     // panel band ends cached in LDS (n <= 8192)
constexpr int kCholLd = kCholWS + 1;
constexpr size_t kCholLds = (size_t)kCholWS * kCholLd * sizeof(double);

__device__ __forceinline__ double& Wn(double* win, int i, int j) {
  return win[(i & (kCholWS - 1)) * kCholLd + (j & (kCholWS - 1))];
}

// 1/sqrt(x): v_rsq_f64 and one Newton step in FMA form, y (1.5 - x y^2 / 2) (relative error ~1e-14, far
// inside the solver's parity tolerances; the pivot chain of the panel factorisation runs through it).
__device__ __forceinline__ double rsq_nr1(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  const double e = fma(-(h * y), y, 0.5);
  return fma(y, e, y);
}

// Wave-uniform broadcast of lane `l`'s double (v_readlane pair: no LDS round trip).
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// The lane id through an opaque move: comparisons against it inside a loop are not hoisted out as
// loop-invariant 64-bit lane masks (which would otherwise pile up in SGPRs and spill).
__device__ __forceinline__ int opaque_lane() {
  int v = __lane_id();
  asm volatile("v_mov_b32 %0, %0" : "+v"(v));
  return v;
}


// Unblocked factorisation of the w x w diagonal block held column-per-lane (lanes 0..w-1, col[r] =
// A[r][lane] for r <= lane), broadcasts by v_readlane.  `bad` is set on a non-positive pivot.
__device__ __forceinline__ void chol_diag16(double (&col)[kCholNb], int w, int lane, bool& bad) {
#pragma unroll
  for (int j = 0; j < kCholNb; ++j) {
    if (j < w) {
      const double piv = readlane_d(col[j], j);
      if (!(piv > 0.0)) bad = true;
      const double ujj = sqrt(piv);
      const double inv = 1.0 / ujj;
      col[j] = (lane == j) ? ujj : (lane > j ? col[j] * inv : col[j]);
#pragma unroll
      for (int r = j + 1; r < kCholNb; ++r) {
        if (r < w) {
          const double ujr = readlane_d(col[j], r);
          if (lane >= r) col[r] -= ujr * col[j];
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Right-looking forward substitution of one 16-row column with U11^T (U11 and 1/diag in LDS).
__device__ __forceinline__ void chol_trsm16(double (&a)[kCholNb], const double (*U11)[kCholNb + 1],
                                            const double* rdiag, int w) {
#pragma unroll
  for (int m = 0; m < kCholNb; ++m) {
    if (m < w) {
      a[m] *= rdiag[m];
#pragma unroll
      for (int j = m + 1; j < kCholNb; ++j)
        if (j < w) a[j] -= U11[m][j] * a[m];
    }
    __builtin_amdgcn_sched_barrier(0);   // keep each step's LDS reads local (no 120-load hoist)
  }
}

// Back substitution U x = y.  U rows in global A (band end per panel), 1/U_jj in rdg, forward solution
// in y (global); the solution goes to xs (LDS, n doubles) and y.  Blocked by 16 from the end; the
// 16x16 triangle runs in one wave with readlane broadcasts.
// kc0 < n: the arrowhead layout of k_cholesky_global (row panel pk's columns [kb + w, panel_jend[npanel + pk])
// then [max(kc0, kb + w), n)).
__device__ __noinline__ void chol_backsub(const double* A, const double* rdg, double* y, double* xs, int n,
                                          const int32_t* panel_jend, int kc0) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
  const int npanel = (n + kCholNb - 1) / kCholNb;
  __shared__ double rpart[kCholNb];
  for (int pk = npanel - 1; pk >= 0; --pk) {
    const int kb = pk * kCholNb;
    const int w = min(kCholNb, n - kb);
    const int c0 = kb + w;
    const int bend = kc0 < n ? max(c0, panel_jend[npanel + pk]) : panel_jend[pk];
    const int klo = kc0 < n ? max(kc0, c0) : n;
    const int m1 = bend - c0, m = m1 + (n - klo);
    for (int r = wave; r < w; r += nwaves) {
      double s = 0.0;
      for (int ci = lane; ci < m; ci += 64) {
        const int j = ci < m1 ? c0 + ci : klo + (ci - m1);
        s += A[(size_t)(kb + r) * n + j] * xs[j];
      }
      s = wave_sum(s);
      if (lane == 0) rpart[r] = s;
    }
    lds_barrier();
    if (wave == 0) {
      double row[kCholNb];
#pragma unroll
      for (int c = 0; c < kCholNb; ++c)
        row[c] = (lane < w && c < w && c > lane) ? A[(size_t)(kb + lane) * n + kb + c] : 0.0;
      const double rd = lane < w ? rdg[kb + lane] : 0.0;
      double v = lane < w ? y[kb + lane] - rpart[lane] : 0.0;
#pragma unroll
      for (int j = kCholNb - 1; j >= 0; --j) {
        if (j < w) {
          const double xj = readlane_d(v * rd, j);
          if (lane == j) v = xj;
          else if (lane < j) v -= row[j] * xj;
        }
      }
      if (lane < w) {
        xs[kb + lane] = v;
        y[kb + lane] = v;
      }
    }
    lds_barrier();
  }
}

// Candidate camera poses x+ = Plus(x, -S x_c) for every frame, FrameDistance model / candidate terms.
template <int NT>
__device__ __forceinline__ void chol_candidates(const Dev& d, const double* y, int fail, int tmo = 0) {
  const LmState* st = d.st;
  __shared__ double red[4 * NT / 64];
  const int tid = threadIdx.x;
  const int cur = st->cur, nxt = cur ^ 1;
  double step2 = 0.0, candx2 = 0.0, model = 0.0, candcost = 0.0;
  for (int f = tid; f < d.F; f += blockDim.x) {
    const double* q = d.q[cur] + 4 * f;
    const double* t = d.t[cur] + 3 * f;
    double* qn = d.q[nxt] + 4 * f;
    double* tn = d.t[nxt] + 3 * f;
    const int b = d.frame_block[f];
    double qq[4] = {q[0], q[1], q[2], q[3]}, tt[3] = {t[0], t[1], t[2]};
    if (b >= 0) {
      if (d.rot_free[f]) {
        double dl[3];
        for (int a = 0; a < 3; ++a) dl[a] = -y[6 * b + a] * d.scale_c[6 * b + a];
        QuatPlus(q, dl, qq);
        for (int a = 0; a < 4; ++a) {
          step2 += (qq[a] - q[a]) * (qq[a] - q[a]);
          candx2 += qq[a] * qq[a];
        }
      }
      if (d.trans_free[f]) {
        for (int a = 0; a < 3; ++a) {
          tt[a] = t[a] - y[6 * b + 3 + a] * d.scale_c[6 * b + 3 + a];
          step2 += (tt[a] - t[a]) * (tt[a] - t[a]);
          candx2 += tt[a] * tt[a];
        }
      }
    }
    for (int a = 0; a < 4; ++a) qn[a] = qq[a];
    for (int a = 0; a < 3; ++a) tn[a] = tt[a];
  }
  __syncthreads();
  for (int dd = tid; dd < d.D; dd += blockDim.x) {
    const int fa = d.fd_a[dd], fb = d.fd_b[dd];
    const int ba = d.frame_block[fa], bb = d.frame_block[fb];
    const double* Jd = d.fd_J + 6 * dd;
    double m = 0.0;
    for (int j = 0; j < 3; ++j) {
      if (ba >= 0) m += Jd[j] * d.scale_c[6 * ba + 3 + j] * (-y[6 * ba + 3 + j]);
      if (bb >= 0) m += Jd[3 + j] * d.scale_c[6 * bb + 3 + j] * (-y[6 * bb + 3 + j]);
    }
    model -= m * (d.fd_r[dd] + 0.5 * m);
    const double* ta = d.t[nxt] + 3 * fa;
    const double* tb = d.t[nxt] + 3 * fb;
    const double e0 = ta[0] - tb[0], e1 = ta[1] - tb[1], e2 = ta[2] - tb[2];
    const double r = 0.1 * (sqrt(e0 * e0 + e1 * e1 + e2 * e2) - d.fd_target);
    double rho0, rho1;
    Cauchy(r * r, d.fd_b2, d.fd_inv_b2, &rho0, &rho1);
    candcost += 0.5 * rho0;
  }
  double sums[4] = {step2, candx2, model, candcost};
  block_sum_multi<NT, 4>(sums, red);
  step2 = sums[0];
  candx2 = sums[1];
  model = sums[2];
  candcost = sums[3];
  if (tid == 0) {
    d.xchg_chol[kCStep2] = step2;
    d.xchg_chol[kCCandX2] = candx2;
    d.xchg_chol[kCModel] = model;
    d.xchg_chol[kCCandCost] = candcost;
    d.xchg_chol[kCFail] = fail ? 1.0 : 0.0;
    d.xchg_chol[kCTimeout] = tmo ? 1.0 : 0.0;
  }
}

// The tiled Cholesky's candidate pass with its operands staged in LDS: waves the back substitution does not
// use load them (poses at x[cur], frame blocks and freedom flags, the column scales, the FrameDistance
// pairs, Jacobians and residuals) while it runs, so the pass after it is LDS-only but for the candidate
// stores.  Same arithmetic and summation order as chol_candidates.
constexpr int kCandMax = 1024;   // frames / FrameDistance residuals staged (more: chol_candidates)
struct CandLds {
  double *q, *t, *sc, *J, *r, *tn;
  int *fb, *fl, *fa, *fbb, *ba, *bb;
  static size_t bytes(int F, int D, int n) {
    return (size_t)(7 * F + n + 7 * D + 3 * F) * sizeof(double) + (size_t)(2 * F + 4 * D) * sizeof(int);
  }
  __device__ void carve(double* base, int F, int D, int n) {
    q = base; t = q + 4 * F; sc = t + 3 * F; J = sc + n; r = J + 6 * D; tn = r + D;
    fb = reinterpret_cast<int*>(tn + 3 * F); fl = fb + F; fa = fl + F; fbb = fa + D; ba = fbb + D; bb = ba + D;
  }
};

__device__ __forceinline__ void cand_prefetch(const Dev& d, const CandLds& c, int cur, int i0, int ni) {
  for (int f = i0; f < d.F; f += ni) {
    const int b = d.frame_block[f];
    c.fb[f] = b;
    c.fl[f] = (d.rot_free[f] ? 1 : 0) | (d.trans_free[f] ? 2 : 0);
    for (int a = 0; a < 4; ++a) c.q[4 * f + a] = d.q[cur][4 * f + a];
    for (int a = 0; a < 3; ++a) c.t[3 * f + a] = d.t[cur][3 * f + a];
  }
  for (int i = i0; i < d.n; i += ni) c.sc[i] = d.scale_c[i];
  for (int e = i0; e < d.D; e += ni) {
    const int fa = d.fd_a[e], fb = d.fd_b[e];
    c.fa[e] = fa;
    c.fbb[e] = fb;
    c.ba[e] = d.frame_block[fa];
    c.bb[e] = d.frame_block[fb];
    for (int j = 0; j < 6; ++j) c.J[6 * e + j] = d.fd_J[6 * e + j];
    c.r[e] = d.fd_r[e];
  }
}

template <int NT>
__device__ __forceinline__ void chol_candidates_lds(const Dev& d, const double* y, int fail, const CandLds& c,
                                                    int cur, int tmo) {
  __shared__ double red[4 * NT / 64];
  const int tid = threadIdx.x;
  const int nxt = cur ^ 1;
  double step2 = 0.0, candx2 = 0.0, model = 0.0, candcost = 0.0;
  for (int f = tid; f < d.F; f += NT) {
    const double* q = c.q + 4 * f;
    const double* t = c.t + 3 * f;
    double* qn = d.q[nxt] + 4 * f;
    double* tn = d.t[nxt] + 3 * f;
    const int b = c.fb[f];
    const int fl = c.fl[f];
    double qq[4] = {q[0], q[1], q[2], q[3]}, tt[3] = {t[0], t[1], t[2]};
    if (b >= 0) {
      if (fl & 1) {
        double dl[3];
        for (int a = 0; a < 3; ++a) dl[a] = -y[6 * b + a] * c.sc[6 * b + a];
        QuatPlus(q, dl, qq);
        for (int a = 0; a < 4; ++a) {
          step2 += (qq[a] - q[a]) * (qq[a] - q[a]);
          candx2 += qq[a] * qq[a];
        }
      }
      if (fl & 2) {
        for (int a = 0; a < 3; ++a) {
          tt[a] = t[a] - y[6 * b + 3 + a] * c.sc[6 * b + 3 + a];
          step2 += (tt[a] - t[a]) * (tt[a] - t[a]);
          candx2 += tt[a] * tt[a];
        }
      }
    }
    for (int a = 0; a < 4; ++a) qn[a] = qq[a];
    for (int a = 0; a < 3; ++a) {
      tn[a] = tt[a];
      c.tn[3 * f + a] = tt[a];
    }
  }
  __syncthreads();
  for (int dd = tid; dd < d.D; dd += NT) {
    const int fa = c.fa[dd], fb = c.fbb[dd];
    const int ba = c.ba[dd], bb = c.bb[dd];
    const double* Jd = c.J + 6 * dd;
    double m = 0.0;
    for (int j = 0; j < 3; ++j) {
      if (ba >= 0) m += Jd[j] * c.sc[6 * ba + 3 + j] * (-y[6 * ba + 3 + j]);
      if (bb >= 0) m += Jd[3 + j] * c.sc[6 * bb + 3 + j] * (-y[6 * bb + 3 + j]);
    }
    model -= m * (c.r[dd] + 0.5 * m);
    const double* ta = c.tn + 3 * fa;
    const double* tb = c.tn + 3 * fb;
    const double e0 = ta[0] - tb[0], e1 = ta[1] - tb[1], e2 = ta[2] - tb[2];
    const double r = 0.1 * (sqrt(e0 * e0 + e1 * e1 + e2 * e2) - d.fd_target);
    double rho0, rho1;
    Cauchy(r * r, d.fd_b2, d.fd_inv_b2, &rho0, &rho1);
    candcost += 0.5 * rho0;
  }
  double sums[4] = {step2, candx2, model, candcost};
  block_sum_multi<NT, 4>(sums, red);
  if (tid == 0) {
    d.xchg_chol[kCStep2] = sums[0];
    d.xchg_chol[kCCandX2] = sums[1];
    d.xchg_chol[kCModel] = sums[2];
    d.xchg_chol[kCCandCost] = sums[3];
    d.xchg_chol[kCFail] = fail ? 1.0 : 0.0;
    d.xchg_chol[kCTimeout] = tmo ? 1.0 : 0.0;
  }
}

// Diagnostic stamps (SG_STAMP=1 builds of the launch only): thread 0 accumulates s_memtime deltas per phase
// in registers (a global read-modify-write here would wait on every outstanding load) and adds them to
// d.stamps once at the end.
#define SG_STAMP_AT(slot)                                                        \
  asm volatile("" ::: "memory");  /* phase boundary: same code motion with or without stamps */ \
  if (kStamp && threadIdx.x == 0) {                                               \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                 \
    stamp_acc[slot] += now_ - last_stamp;                                         \
    last_stamp = now_;                                                            \
  }
#define SG_STAMP_FLUSH()                                                         \
  if (kStamp && threadIdx.x == 0) {                                               \
    for (int s_ = 0; s_ < 16; ++s_) d.stamps[s_] += stamp_acc[s_];                 \
  }

// Back substitution of the window path from x_p = z_p - W_p x_rest (W = U11^-1 U12 and z = U11^-1 y per
// panel, stored over the U rows of A and over y): one mat-vec per panel, two rows per wave.  The operands of
// the next kBsDepth panels are in flight in registers (a ring, statically indexed by an unrolled loop), so
// a panel step waits on LDS and the DPP reduction, not on a global load.
#ifndef SG_BS_DEPTH
#define SG_BS_DEPTH 4   // measured best of 4 / 8 / 12 (fewer loads queued per wave)
#endif
constexpr int kBsDepth = SG_BS_DEPTH;
struct BsOps {
  double2 w[2];   // rows kb + 2 wave + h, columns kb + 16 + 2 lane + {0, 1}
  double2 z;      // z of the two rows
  int jend;
};
__device__ __forceinline__ void chol_bs_load(const double* Wm, const double* z, int n, const int* jend_sh, int pk,
                                             int wave, int lane, BsOps& o) {
  // Branch-free 16-byte loads: every call issues the same three global loads (clamped addresses; entries
  // outside the band are masked at the use), so the compiler's vmcnt accounting stays exact and a panel
  // step waits only on the loads issued kBsDepth steps earlier.  n = 6 x blocks and kb are even, so a
  // column pair never straddles n or the (16-aligned) band end.
  const bool pv = pk >= 0;
  const int kb = (pv ? pk : 0) * kCholNb;
  o.jend = pv ? jend_sh[pv ? pk : 0] : 0;
  const int r0 = kb + 2 * wave;
  const int c = kb + kCholNb + 2 * lane;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const bool rin = pv && r0 + h < n;
    o.w[h] = *reinterpret_cast<const double2*>(Wm + ((rin && c < n) ? (size_t)(r0 + h) * n + c : 0));
  }
  o.z = *reinterpret_cast<const double2*>(z + ((pv && r0 < n) ? r0 : 0));
}

template <bool kStamp>
__device__ __forceinline__ void chol_backsub_w(const double* Wm, const double* z, double* xs, int n,
                                               const int* jend_sh, const int32_t* panel_jend,
                                               unsigned long long (&stamp_acc)[16], unsigned long long& last_stamp) {
  (void)panel_jend;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  static_assert(kCholThreads / 64 * 2 == kCholNb, "two panel rows per wave");
  const int npanel = (n + kCholNb - 1) / kCholNb;
  BsOps ring[kBsDepth];
#pragma unroll
  for (int s = 0; s < kBsDepth; ++s) chol_bs_load(Wm, z, n, jend_sh, npanel - 1 - s, wave, lane, ring[s]);
  for (int base = npanel - 1; base >= 0; base -= kBsDepth) {
#pragma unroll
    for (int s = 0; s < kBsDepth; ++s) {
      const int pk = base - s;   // workgroup-uniform
      const BsOps cur = ring[s];
      chol_bs_load(Wm, z, n, jend_sh, pk - kBsDepth, wave, lane, ring[s]);   // unconditional: exact vmcnt
      if (pk >= 0) {
        const int kb = pk * kCholNb;
        const int c = kb + kCholNb + 2 * lane;
        const double2 xv = *reinterpret_cast<const double2*>(xs + c);   // inside the LDS window
        const bool in = c < cur.jend;
        double sv[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const double acc = (in ? cur.w[h].x : 0.0) * (in ? xv.x : 0.0) + (in ? cur.w[h].y : 0.0) * (in ? xv.y : 0.0);
          if (h == 0) { SG_STAMP_AT(11) }
          sv[h] = wave_sum_full(acc);
        }
        SG_STAMP_AT(12)
        if (lane == 0) {
          const int r0 = kb + 2 * wave;
          if (r0 < n) xs[r0] = cur.z.x - sv[0];
          if (r0 + 1 < n) xs[r0 + 1] = cur.z.y - sv[1];
        }
        lds_barrier();
        SG_STAMP_AT(13)
      }
    }
  }
}

// Window path: the active band lives in LDS (132 KiB) together with the rhs ring; finished panel rows and
// 1/U_jj go to global memory for the back substitution.  Barriers between phases are LDS-only, so the
// global writes and the prefetch of the next window columns overlap the factorisation.
// W / z of one finished panel (back-substitution operands, see chol_backsub_w): lane (wave wv0.., lane)
// solves U11 t = U12[:, c] for one column c of the panel's band, one extra lane solves U11 z = y_panel.
// U12 is read from the LDS window (the panel's rows stay there until the next panel's slide), U11 and 1/U_jj
// from the panel's LDS copies.
__device__ __forceinline__ void chol_panel_w(const double* win, const double* u11, const double* pinv,
                                             const double* ypan, int kb, int w, int jend, int n, int wi,
                                             double* __restrict__ S, double* __restrict__ y) {
  const int nc = jend - (kb + kCholNb);   // band columns right of the panel (<= kCholWS - kCholNb)
  const bool isz = wi == kCholWS - kCholNb;
  const int c = kb + kCholNb + wi;
  if (!(wi < nc || isz)) return;
  double t[kCholNb];
  // unconditional loads from a lane-selected address (window column or the panel rhs), all in flight
  // together: per-lane branches here serialise 16 LDS round trips on the critical path of phase (a)
  const double* base = isz ? ypan : win + (c & (kCholWS - 1));
#pragma unroll
  for (int r = 0; r < kCholNb; ++r) t[r] = base[isz ? r : ((kb + r) & (kCholWS - 1)) * kCholLd];
  // U11 columns (rows above the diagonal) and 1/U_kk stream through a 3-deep register ring, column k-2
  // issued before step k's FMAs (scheduling barriers keep the loads ahead of their use)
  double cb[3][kCholNb], pb[3];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = kCholNb - 1 - q;
#pragma unroll
    for (int r = 0; r < k; ++r) cb[k % 3][r] = u11[k * kCholNb + r];
    pb[k % 3] = pinv[k];
  }
#pragma unroll
  for (int r = 0; r < kCholNb; ++r) t[r] = (isz || r < w) ? t[r] : 0.0;
#pragma unroll
  for (int k = kCholNb - 1; k >= 0; --k) {
    if (k >= 2) {
#pragma unroll
      for (int r = 0; r < k - 2; ++r) cb[(k - 2) % 3][r] = u11[(k - 2) * kCholNb + r];
      pb[(k - 2) % 3] = pinv[k - 2];
    }
    __builtin_amdgcn_sched_barrier(0);
    t[k] *= pb[k % 3];
#pragma unroll
    for (int r = 0; r < k; ++r) t[r] = fma(-cb[k % 3][r], t[k], t[r]);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (isz) {
#pragma unroll
    for (int r = 0; r < kCholNb; ++r)
      if (r < w) y[kb + r] = t[r];
  } else {
#pragma unroll
    for (int r = 0; r < kCholNb; ++r)
      if (r < w) S[(size_t)(kb + r) * n + c] = t[r];
  }
}

// Window path: the active band lives in LDS (132 KiB) together with the rhs ring.  Per 16-row panel:
//   phase A  waves 0-2 factor the panel (diagonal block + off-diagonal columns + rhs in one right-looking
//            pass, see below) while waves 3-4 turn the previous panel into back-substitution operands
//            (W = U11^-1 U12, z = U11^-1 y) and store them to global memory;
//   phase B  all waves apply the trailing update A22 -= U12^T U12 (MFMA f64 tiles) and slide the window.
// Barriers are LDS-only, so global stores and the prefetch of the next window columns stay in flight.
template <bool kStamp>
__global__ __launch_bounds__(kCholThreads) void k_cholesky_window(Dev d, const int32_t* panel_jend, double* rdg) {
  unsigned long long last_stamp = kStamp ? __builtin_amdgcn_s_memtime() : 0ull;
  unsigned long long stamp_acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  LmState* st = d.st;
  if (st->done) return;
  extern __shared__ double win[];
  __shared__ double yw[kCholWS];
  __shared__ double prow[kPanelWaves][2 * kCholNb];   // per panel wave: the next two pivot rows
  __shared__ double pinv[2][kCholNb];                 // 1/U_jj of the current / previous panel
  __shared__ double u11w[2][kCholNb * kCholNb];       // U11 columns of the current / previous panel
  __shared__ double ypan[2][kCholNb];                 // forward-substituted rhs of the panel rows
  __shared__ int jend_sh[kJendSh];
  __shared__ int fail_sh;
  const int n = d.n, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwaves = kCholThreads / 64;
  double* y = d.work;
  if (tid == 0) fail_sh = 0;
  // rhs y = rhs_sub + S g_c (assembled by k_S_reduce); initial 128 x 128 window, all loads issued first
  for (int i = tid; i < min(n, kCholWS); i += kCholThreads) yw[i] = d.xc[i];
  const int n0 = min(n, kCholWS);
  constexpr int kInit = kCholWS * kCholWS / kCholThreads;
  {
    double v[kInit];
#pragma unroll
    for (int q = 0; q < kInit; ++q) {
      const int e = tid + q * kCholThreads, i = e / kCholWS, j = e % kCholWS;
      const bool in = i < n0 && j < n0 && i <= j;
      v[q] = d.S[in ? (size_t)i * n + j : 0];
    }
#pragma unroll
    for (int q = 0; q < kInit; ++q) {
      const int e = tid + q * kCholThreads, i = e / kCholWS, j = e % kCholWS;
      if (i < n0 && j < n0 && i <= j) Wn(win, i, j) = v[q];
    }
  }
  const int npanel = (n + kCholNb - 1) / kCholNb;
  for (int p = tid; p < npanel; p += kCholThreads) jend_sh[p] = panel_jend[p];   // npanel <= kJendSh
  __syncthreads();
  SG_STAMP_AT(0)
  const int li = lane & 15, lk = lane >> 4;
  constexpr int kPf = kCholNb * kCholWS / kCholThreads;   // prefetched window elements per thread
  for (int pk = 0; pk < npanel; ++pk) {
    const int kb = pk * kCholNb;
    const int w = min(kCholNb, n - kb);
    const int jend = jend_sh[pk];
    const int buf = pk & 1;
    // prefetch the columns this panel's slide brings in: j in [kb+WS, kb+WS+w), rows kb+w..j
    const int jn0 = kb + kCholWS, jn1 = min(n, jn0 + w);
    double pf[kPf];
#pragma unroll
    for (int q = 0; q < kPf; ++q) {
      const int e = tid + q * kCholThreads;
      const int j = jn0 + e / kCholWS, i = kb + w + e % kCholWS;
      const bool in = j < jn1 && i <= j;
      pf[q] = d.S[in ? (size_t)i * n + j : 0];   // branch-free: the loads stay in flight across phases
    }
    const double pfy = d.xc[min(jn0 + tid, n - 1)];   // rhs entries of the incoming rows (unmodified yet)
    SG_STAMP_AT(14)
    // (a) panel factorisation by kPanelWaves waves: rows kb..kb+15 of the band.  Every panel wave holds
    // the 16 diagonal-block columns in lanes 0..15 (factored redundantly, so no cross-wave sync) and 48
    // off-diagonal columns in lanes 16..63; the diagonal block, the TRSM of the off-diagonal columns and
    // the rhs forward step run as one right-looking pass.  Row j of the diagonal block is broadcast
    // through a per-wave LDS row (one wave: the LDS queue orders write before read, no barrier).  Rows
    // past n are padded with identity so the unrolled loop has no branches.
    if (wave < kPanelWaves) {
      const int lane = opaque_lane();
      const int slot = lane < kCholNb ? lane : kCholNb + (64 - kCholNb) * wave + (lane - kCholNb);
      const int c = kb + slot;
      const bool v = slot < kCholWS && c < jend;
      const bool isy = slot == kCholWS;   // the rhs rides as an augmented column in an otherwise idle lane
      double* prw = prow[wave];
      double ca[kCholNb];
      // one unconditional LDS load per row from a lane-selected address (window column or rhs ring), all
      // issued before the first use: per-lane branches here would serialise 16 LDS round trips
      const double* col0 = isy ? &yw[0] : &Wn(win, 0, c);
      const int rstride = isy ? 1 : kCholLd;
#pragma unroll
      for (int r = 0; r < kCholNb; ++r) ca[r] = col0[((kb + r) & (kCholWS - 1)) * rstride];
#pragma unroll
      for (int r = 0; r < kCholNb; ++r) asm volatile("" : "+v"(ca[r]));
      SG_STAMP_AT(15)
      // Row selection as per-lane bit sets (bit r: keep row r / identity-pad row r), applied with opaque
      // v_bfe_i32 masks: written as selects, the compiler turns this into 16 divergent branches (~2k cycles).
      {
        const unsigned real_rows = (w >= kCholNb) ? 0xFFFFu : ((1u << w) - 1u);
        const unsigned upto = slot >= kCholNb - 1 ? 0xFFFFu : ((2u << slot) - 1u);   // rows r <= slot
        unsigned keepbits = isy ? real_rows : (v ? (real_rows & upto) : 0u);
        unsigned onebits = (!isy && slot < kCholNb && slot >= w) ? (1u << slot) : 0u;
        asm volatile("" : "+v"(keepbits), "+v"(onebits));
        const unsigned long long kOneBits = 0x3FF0000000000000ull;
#pragma unroll
        for (int r = 0; r < kCholNb; ++r) {
          int km, om;
          asm volatile("v_bfe_i32 %0, %1, %2, 1" : "=v"(km) : "v"(keepbits), "n"(r));
          asm volatile("v_bfe_i32 %0, %1, %2, 1" : "=v"(om) : "v"(onebits), "n"(r));
          const unsigned long long b = (unsigned long long)__double_as_longlong(ca[r]);
          ca[r] = __longlong_as_double((long long)((b & (unsigned long long)(long long)km) |
                                                   (kOneBits & (unsigned long long)(long long)om)));
        }
      }
      bool bad = false;
      SG_STAMP_AT(1)
      // Right-looking steps, two pivots per LDS broadcast: rows j and j+1 of the diagonal block arrive
      // together; every lane derives row j+1 after pivot j itself (wave-uniform values, 14 FMAs) instead of
      // waiting for a second round trip.  Pivot j scales row j by 1/U_jj and updates every entry below with
      // A[r][c] -= A[j][r] (A[j][c] / A_jj) (one FMA per entry); pivot j+1 likewise.  Rows j+2 and j+3 are
      // updated first and posted while the remaining updates run.
      double u0[kCholNb], u1[kCholNb];
      double* prw2 = prw + kCholNb;
      if (lane < kCholNb) {
        prw[lane] = ca[0];
        prw2[lane] = ca[1];
      }
#pragma unroll
      for (int r = 0; r < kCholNb; ++r) {
        u0[r] = prw[r];
        u1[r] = prw2[r];
      }
#pragma unroll
      for (int j = 0; j < kCholNb; j += 2) {
        const double p0 = u0[j];
        bad |= !(p0 > 0.0);
        const double i0 = rsq_nr1(p0);
        const double r0 = i0 * i0;                       // 1 / A_jj
        const double w1 = u0[j + 1] * r0;
        double v1[kCholNb];                              // row j+1 after pivot j
#pragma unroll
        for (int r = j + 1; r < kCholNb; ++r) v1[r] = fma(-w1, u0[r], u1[r]);
        const double p1 = v1[j + 1];
        bad |= !(p1 > 0.0);
        const double i1 = rsq_nr1(p1);
        const double r1 = i1 * i1;
        const double aj = ca[j];
        const double t0 = aj * r0;
        ca[j] = aj * i0;
        const double aj1 = fma(-u0[j + 1], t0, ca[j + 1]);
        const double t1 = aj1 * r1;
        ca[j + 1] = aj1 * i1;
        if (wave == 0 && lane == 0) {
          pinv[buf][j] = i0;
          pinv[buf][j + 1] = i1;
        }
        if (j + 2 < kCholNb) {
          ca[j + 2] = fma(-v1[j + 2], t1, fma(-u0[j + 2], t0, ca[j + 2]));
          ca[j + 3] = fma(-v1[j + 3], t1, fma(-u0[j + 3], t0, ca[j + 3]));
          if (lane < kCholNb) {                          // the next two pivot rows
            prw[lane] = ca[j + 2];
            prw2[lane] = ca[j + 3];
          }
        }
#pragma unroll
        for (int r = j + 4; r < kCholNb; ++r) ca[r] = fma(-v1[r], t1, fma(-u0[r], t0, ca[r]));
        // materialise this step's updates here (otherwise they are sunk into later steps and spill)
#pragma unroll
        for (int r = j; r < kCholNb; ++r) asm volatile("" : "+v"(ca[r]));
        if (j + 2 < kCholNb) {
#pragma unroll
          for (int r = j + 2; r < kCholNb; ++r) {
            u0[r] = prw[r];
            u1[r] = prw2[r];
          }
        }
      }
      SG_STAMP_AT(3)
      // trailing columns' panel rows -> LDS; the panel's U11 and 1/U_jj (wave 0) and forward-substituted rhs
      // (the rhs lane) for the W / z pass and the trailing rhs update
      // (one divergent region per destination; rows r >= w of the last panel land in ring slots of retired
      // rows below the previous panel, which nothing reads again)
      const bool trail = v && lane >= kCholNb;
      if (trail) {
#pragma unroll
        for (int r = 0; r < kCholNb; ++r) Wn(win, kb + r, c) = ca[r];
      }
      if (isy) {
#pragma unroll
        for (int r = 0; r < kCholNb; ++r) ypan[buf][r] = ca[r];
      }
      if (wave == 0) {
        if (lane < kCholNb) {
#pragma unroll
          for (int r = 0; r < kCholNb; ++r) u11w[buf][lane * kCholNb + r] = ca[r];
        }
        if (lane == 0 && bad) fail_sh = 1;
      }
    } else if (pk > 0 && wave < kPanelWaves + 2) {
      // (a') the previous panel's back-substitution operands, off the critical path
      const int pb = pk - 1;
      chol_panel_w(win, u11w[buf ^ 1], pinv[buf ^ 1], ypan[buf ^ 1], pb * kCholNb, min(kCholNb, n - pb * kCholNb),
                   jend_sh[pb], n, (wave - kPanelWaves) * 64 + lane, d.S, y);
    }
    lds_barrier();
    SG_STAMP_AT(2)
    // (b) rhs of the trailing rows, y_c -= sum_r U[r][c] ytilde_r (one thread per band column), and the
    // trailing update A22 -= U12^T U12 on the band, 16x16 MFMA tiles (upper tiles only)
    if (tid < kCholWS - kCholNb) {
      const int c = kb + kCholNb + tid;
      if (c < jend) {
        double s0 = 0.0;
#pragma unroll
        for (int r = 0; r < kCholNb; ++r) s0 += (r < w ? Wn(win, kb + r, c) : 0.0) * ypan[buf][r];
        yw[c & (kCholWS - 1)] -= s0;
      }
    }
    const int m = jend - (kb + w);
    const int T = (m + 15) >> 4;
    const int ntiles = T * (T + 1) / 2;
    for (int tile = wave; tile < ntiles; tile += nwaves) {
      int ti = 0, rem = tile;
      while (rem >= T - ti) { rem -= T - ti; ++ti; }
      const int tj = ti + rem;
      const int i0 = kb + w + 16 * ti, j0 = kb + w + 16 * tj;
      f64x4 acc;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int row = i0 + lk + 4 * qq, col = j0 + li;
        const double wv = Wn(win, row, col);   // ring index: always a valid address
        acc[qq] = (row < jend && col < jend && row <= col) ? wv : 0.0;
      }
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int k = kb + 4 * s4 + lk;
        const bool kin = (4 * s4 + lk) < w;
        const double wa = Wn(win, k, i0 + li), wb = Wn(win, k, j0 + li);
        const double av = (kin && i0 + li < jend) ? -wa : 0.0;
        const double bv = (kin && j0 + li < jend) ? wb : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int row = i0 + lk + 4 * qq, col = j0 + li;
        if (row < jend && col < jend && row <= col) Wn(win, row, col) = acc[qq];
      }
    }
    SG_STAMP_AT(4)
    // (c) slide the window: columns [kb + WS, kb + WS + w) replace the departed rows/columns.  Disjoint
    // from everything the trailing update touches (columns < jend <= kb + WS), so no barrier between.
#pragma unroll
    for (int q = 0; q < kPf; ++q) {
      const int e = tid + q * kCholThreads;
      const int j = jn0 + e / kCholWS, i = kb + w + e % kCholWS;
      if (j < jn1 && i <= j) Wn(win, i, j) = pf[q];
    }
    if (tid < jn1 - jn0) yw[(jn0 + tid) & (kCholWS - 1)] = pfy;
    lds_barrier();
    SG_STAMP_AT(5)
  }
  // the last panel's operands
  if (wave >= kPanelWaves && wave < kPanelWaves + 2) {
    const int pb = npanel - 1;
    chol_panel_w(win, u11w[pb & 1], pinv[pb & 1], ypan[pb & 1], pb * kCholNb, min(kCholNb, n - pb * kCholNb),
                 jend_sh[pb], n, (wave - kPanelWaves) * 64 + lane, d.S, y);
  }
  SG_STAMP_AT(8)
  __syncthreads();   // global W rows / z visible to every wave
  SG_STAMP_AT(9)
  double* xs = win;  // the window is free now: the solution lives in LDS
  chol_backsub_w<kStamp>(d.S, y, xs, n, jend_sh, panel_jend, stamp_acc, last_stamp);
  SG_STAMP_AT(10)
  for (int i = tid; i < n; i += kCholThreads) {
    d.xc[i] = xs[i];
    y[i] = xs[i];
  }
  __syncthreads();
  SG_STAMP_AT(6)
  chol_candidates<kCholThreads>(d, xs, fail_sh);
  SG_STAMP_AT(7)
  SG_STAMP_FLUSH()
}

// Global-memory path for bands wider than the LDS window (a dense S: free intrinsics couple every frame).
// Right-looking over 16-row panels: wave 0 factors the diagonal block, a thread per column does the panel's
// TRSM, and the trailing update A_IJ -= U_KI^T U_KJ runs over 16 x 16 tiles (I <= J), four
// v_mfma_f64_16x16x4f64 a tile with the tile in the accumulator, a wave per tile.  kStage: the panel's
// factored rows are staged in LDS (after xs, pitch n) so the update reads its operands from LDS; the launch
// takes the <false> instance when 17 n doubles do not fit.
// With free intrinsics S is an arrowhead: the frame columns keep their band and only the nk intrinsics columns
// are dense, so a panel's trailing columns are [kb + w, bend) (the frame band end, panel_jend[npanel + pk])
// followed by [max(kc0, kb + w), n); the factor has no fill outside them (a frame column's envelope starts
// after the panel's rows).  The update runs over that compact index space (ci -> column).
template <bool kStage>
__global__ __launch_bounds__(kCholThreads) void k_cholesky_global(Dev d, const int32_t* panel_jend, double* rdg) {
  LmState* st = d.st;
  if (st->done) return;
  extern __shared__ double xs[];   // n doubles: back-substitution solution (then the staged panel rows)
  const int n = d.n, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lk = lane >> 4, li = lane & 15;
  const int nwaves = kCholThreads / 64;
  double* A = d.S;
  double* y = d.work;
  __shared__ double U11[kCholNb][kCholNb + 1];
  __shared__ double rdiag[kCholNb];
  __shared__ int fail_sh;
  if (tid == 0) fail_sh = 0;
  for (int i = tid; i < n; i += kCholThreads) y[i] = d.xc[i];   // assembled rhs (k_S_reduce)
  __syncthreads();
  const int npanel = (n + kCholNb - 1) / kCholNb;
  for (int pk = 0; pk < npanel; ++pk) {
    const int kb = pk * kCholNb;
    const int w = min(kCholNb, n - kb);
    const int jmax = panel_jend[pk];
    if (wave == 0) {
      double col[kCholNb];
#pragma unroll
      for (int r = 0; r < kCholNb; ++r) col[r] = (lane < w && r <= lane) ? A[(size_t)(kb + r) * n + kb + lane] : 0.0;
      bool bad = false;
      chol_diag16(col, w, lane, bad);
      if (lane < w) {
#pragma unroll
        for (int r = 0; r < kCholNb; ++r)
          if (r <= lane) {
            A[(size_t)(kb + r) * n + kb + lane] = col[r];
            U11[r][lane] = col[r];
          }
        const double rd = 1.0 / col[lane];
        rdiag[lane] = rd;
        rdg[kb + lane] = rd;
      }
      if (lane == 0 && bad) fail_sh = 1;
    }
    __syncthreads();
    const int c0 = kb + w;
    int m1 = jmax - c0, klo = n;     // trailing columns: [c0, c0 + m1) then [klo, n)
    if (d.nk > 0) {
      m1 = max(0, panel_jend[npanel + pk] - c0);
      klo = max(d.kc0, c0);
    }
    const int m = m1 + (n - klo);
    auto colof = [&](int ci) -> size_t { return (size_t)(ci < m1 ? c0 + ci : klo + (ci - m1)); };
    double* P = xs + n;              // staged panel rows: P[r n + ci], column colof(ci)
    // U_K row r, trailing column ci (LDS when staged; never a pointer that may be either: flat accesses)
    auto U = [&](int r, int ci) -> double {
      if constexpr (kStage) return P[r * n + ci];
      else return A[(size_t)(kb + r) * n + colof(ci)];
    };
    for (int ci = tid; ci < m + 1; ci += kCholThreads) {
      const bool isy = ci == m;
      double a[kCholNb];
#pragma unroll
      for (int r = 0; r < kCholNb; ++r) a[r] = (r < w) ? (isy ? y[kb + r] : A[(size_t)(kb + r) * n + colof(ci)]) : 0.0;
      chol_trsm16(a, U11, rdiag, w);
#pragma unroll
      for (int r = 0; r < kCholNb; ++r)
        if (r < w) {
          if (isy) {
            y[kb + r] = a[r];
          } else {
            A[(size_t)(kb + r) * n + colof(ci)] = a[r];
            if constexpr (kStage) P[r * n + ci] = a[r];
          }
        }
    }
    __syncthreads();
    const int T = (m + 15) >> 4;
    const int ntiles = T * (T + 1) / 2;
    // kTU consecutive tiles (row-major over I <= J) a wave at a time: their loads in flight together
    constexpr int kTU = 4;
    for (int t0 = wave * kTU; t0 < ntiles; t0 += nwaves * kTU) {
      int i0[kTU], j0[kTU];
      {
        int ti = 0, rem = t0;
        while (rem >= T - ti) { rem -= T - ti; ++ti; }
#pragma unroll
        for (int u = 0; u < kTU; ++u) {
          const bool ok = t0 + u < ntiles;
          i0[u] = ok ? 16 * ti : m;   // an absent tile is masked out by row < m
          j0[u] = ok ? 16 * (ti + rem) : m;
          if (++rem >= T - ti) { ++ti; rem = 0; }
        }
      }
      f64x4 acc[kTU];
#pragma unroll
      for (int u = 0; u < kTU; ++u)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int row = i0[u] + lk + 4 * qq, col = j0[u] + li;
          acc[u][qq] = (row < m && col < m && row <= col) ? A[colof(row) * n + colof(col)] : 0.0;
        }
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int r = 4 * s4 + lk;
        const bool kin = r < w;
#pragma unroll
        for (int u = 0; u < kTU; ++u) {
          const double av = (kin && i0[u] + li < m) ? -U(r, i0[u] + li) : 0.0;
          const double bv = (kin && j0[u] + li < m) ? U(r, j0[u] + li) : 0.0;
          acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[u], 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < kTU; ++u)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int row = i0[u] + lk + 4 * qq, col = j0[u] + li;
          if (row < m && col < m && row <= col) A[colof(row) * n + colof(col)] = acc[u][qq];
        }
    }
    for (int ci = tid; ci < m; ci += kCholThreads) {
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < kCholNb; ++r)
        if (r < w) s += U(r, ci) * y[kb + r];
      y[colof(ci)] -= s;
    }
    __syncthreads();
  }
  chol_backsub(A, rdg, y, xs, n, panel_jend, d.nk > 0 ? d.kc0 : n);
  for (int i = tid; i < n; i += kCholThreads) d.xc[i] = xs[i];
  __syncthreads();
  chol_candidates<kCholThreads>(d, y, fail_sh);
}

// ------------------------------------------------------------------------------------------------
// Tiled band Cholesky — the default reduced-camera solve (SPARSE_SCHUR + CHOLMOD behind slam.cpp:489,
// restated as a dense banded factorisation S = U^T U of 16 x 16 tiles, right-looking, with the band of tile
// columns resident in registers as MFMA accumulators).
//   * 8 waves; wave w owns tile column J = w (mod 8): its tiles (I, J), J - 7 <= I <= J, live in slot I & 7
//     of f64x4 acc[8] (v_mfma_f64_16x16x4f64 C/D layout: lane l holds rows (l >> 4) + 4 q of column l & 15).
//     A column retires when it becomes the diagonal; its wave then loads column J + 8 from S.
//   * One phase (one LDS barrier) per tile row K; every wave, in order:
//       (0) the trailing update of its column by row K-1, A_IJ -= U_{K-1,I}^T U_{K-1,J} (four MFMAs a tile,
//           U_{K-1,I} from LDS), row K first;
//       (1) the TRSM of its row-K tile, U_KJ = Z_K A_KJ (MFMA with Z_K = U_KK^-T), posted to LDS for (0) of
//           the next phase, and its rhs term y_J -= U_KJ^T z_K (per-lane partials);
//       (2) the owner of column K+1 applies row K to D_{K+1} and factors it on the spot with the identity
//           and y_{K+1} as augmented columns (right-looking, two pivots per LDS broadcast), posting Z_{K+1},
//           z_{K+1} = Z_{K+1} y_{K+1} and Z_{K+1}^T z_{K+1} — the critical path of the phase, overlapping
//           every other wave's trailing update;
//       (3) W_KJ = Z_K^T U_KJ (= U_KK^-1 U_KJ) to global memory for the back substitution;
//       (4) the owner reloads.
//   * Back substitution x_K = Z_K^T z_K - sum_d W_{K,K+d} x_{K+d}: wave w forms the d = w + 1 term (W tiles
//     prefetched four rows ahead), one barrier per tile row, every wave sums the partials in the same order.
// Requires a band of at most 8 tiles per tile row (the sliding window's co-visibility band at the configured
// window sizes); wider bands take k_cholesky_global.
constexpr int kTB = 8;                         // band width in tiles = waves
constexpr int kTileThreads = kTB * 64;
constexpr int kTLd = 17;                       // LDS pitch of a 16 x 16 tile
constexpr int kTileMaxNT = 400;                // dynamic LDS: x, z' (16 NT doubles each) + band ends
struct TileShared {
  double Zs[4][16 * kTLd];     // Z_K = U_KK^-T (lower triangular), row-major; 4 deep: the previous owner
  double zK[4][16];            // reads Z_K one phase late.  z_K = Z_K y_K
  double Ur[2][kTB - 1][256];  // row K: U_{K,K+d}, d = 1..7, acc layout
  double Dw[16 * kTLd];        // the owner's diagonal tile (one owner per phase)
  double Yw[16];
  double prw[2 * kCholNb];     // the owner's next two pivot rows
  int fail;
  int tmo;                     // a hand-off wait hit its spin limit (kCTimeout)
  int uflag;                   // look-ahead: the last phase whose owner has posted U_{K,K+1} (Ur[K & 1][0])
  int dflag;                   // Dinv mode: the last phase whose D_K^-1 and z'_K are posted (Dv, zp)
  int uposted;                 // dataflow mode: U tiles posted so far (all rows, monotonic)
  int zflag;                   // dataflow mode: the last K whose Z_K and z_K are posted
  double Dv[16 * kTLd];        // Dinv mode: D_K^-1 = Z_K^T Z_K, row-major
  int simd[kTB];               // SIMD of each wave
  double Id[16 * kTLd];        // the identity (the factor's augmented columns)
};

__device__ __forceinline__ f64x4 mfma_f64_k16(const double (&a)[4], const f64x4& b, f64x4 c) {
#pragma unroll
  for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], c, 0, 0, 0);
  return c;
}

// Sum over the four 16-lane rows (lanes l, l^16, l^32, l^48) by gfx950 permlane swaps; every lane gets
// (v0 + v2) + (v1 + v3), the same bits in each (addition commutes).
__device__ __forceinline__ double sum_rows4(double v) {
  auto a = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
  auto b = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
  const double w = __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
  auto c = __builtin_amdgcn_permlane16_swap(__double2loint(w), __double2loint(w), false, false);
  auto e = __builtin_amdgcn_permlane16_swap(__double2hiint(w), __double2hiint(w), false, false);
  return __hiloint2double(e[0], c[0]) + __hiloint2double(e[1], c[1]);
}

// Row-sum inside each 16-lane row (row_ror butterflies); lane-dependent association, so one fixed lane
// per row consumes it.
__device__ __forceinline__ double row_sum16(double v) {
  v += dpp_d<0x128>(v);   // row_ror:8
  v += dpp_d<0x124>(v);   // row_ror:4
  v += dpp_d<0x122>(v);   // row_ror:2
  v += dpp_d<0x121>(v);   // row_ror:1
  return v;
}

// Tile (I, J) of S in acc layout (entries below the diagonal of a diagonal tile are whatever S holds: the
// factorisation masks them); the identity beyond n (padding rows of the last tile) and zeros for I < 0 come
// from the constants {0, 1} stored after S and its rhs (S[n n + n], S[n n + n + 1]).  The index is selected,
// not the value, so the loads stay in flight until the tile is first used.
// Where a workgroup's tiles come from.  The top half (and the one-workgroup factorisation) reads S as it is;
// the bottom half of the dissected band (k_chol_tiles, blockIdx 1) factors the index-reversed matrix
// P S P (index i -> 16 NT - 1 - i, still banded), whose upper tile (I, J) is the transposed lower tile of S,
// and starts its separator tiles (rows and columns >= sep) and their rhs at zero: the top half holds S there.
// nb: the factored system's order (the frame part, nb = kc0, when the free intrinsics border it: k_chol_border);
// ld: S's pitch (its full order n; the rhs follows S at ld ld, the constants at ld ld + ld).
struct TileSrc {
  int rev;   // 0: S as stored; 1: reversed
  int np;    // 16 NT (padded order)
  int sep;   // first separator tile row (reversed side only; the top half passes NT)
  int nb;    // rows / columns factored
  int ld;    // pitch of S
};

__device__ __forceinline__ f64x4 tile_load(const double* __restrict__ S, int I, int J, int li, int lk,
                                           const TileSrc& ts) {
  f64x4 t;
  const int n = ts.nb, ld = ts.ld;
  const int cz = ld * ld + ld;
  const bool zsep = I >= ts.sep && J >= ts.sep;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int gi = 16 * I + lk + 4 * q, gj = 16 * J + li;
    // source row / column in S's own order (upper triangle: si <= sj for I <= J)
    const int si = ts.rev ? ts.np - 1 - gj : gi, sj = ts.rev ? ts.np - 1 - gi : gj;
    const bool in = I >= 0 && si < n && sj < n && !zsep;
    t[q] = S[in ? si * ld + sj : cz + ((gi == gj && !zsep) ? 1 : 0)];
  }
  return t;
}


// Factor one 16x16 diagonal tile D (upper triangle, pitch kTLd) with the identity (lanes 16-31) and the rhs
// (lane 32) as augmented columns; lanes 0-15 hold the columns of D.  Right-looking, two pivots per LDS
// broadcast (every lane derives pivot row j+1 after pivot j itself).  On return lanes 16-31 hold the columns
// of Z = U^-T and lane 32 holds z = U^-T y.  Returns true on a non-positive pivot.
__device__ __forceinline__ bool tile_factor(const double* D, const double* Yk, const double* Id, double* prw,
                                            double (&ca)[16]) {
  const int lane = opaque_lane();
  const int c = lane & 15;
  const bool isy = lane == 32;
  // D arrives with its lower triangle zeroed and the identity is a constant LDS tile, so every lane just
  // loads its column (no per-element masking on the critical path)
  const double* b0 = isy ? Yk : ((lane >= 16 && lane < 32) ? Id + c : D + c);
  const int rs = isy ? 1 : kTLd;
#pragma unroll
  for (int r = 0; r < kCholNb; ++r) ca[r] = b0[r * rs];
  bool bad = false;
  double u0[kCholNb], u1[kCholNb];
  double* prw2 = prw + kCholNb;
  if (lane < kCholNb) {
    prw[lane] = ca[0];
    prw2[lane] = ca[1];
  }
#pragma unroll
  for (int r = 0; r < kCholNb; ++r) {
    u0[r] = prw[r];
    u1[r] = prw2[r];
  }
#pragma unroll
  for (int j = 0; j < kCholNb; j += 2) {
    const double p0 = u0[j];
    bad |= !(p0 > 0.0);
    const double i0 = rsq_nr1(p0);
    const double r0 = i0 * i0;
    const double w1 = u0[j + 1] * r0;
    double v1[kCholNb];
#pragma unroll
    for (int r = j + 1; r < kCholNb; ++r) v1[r] = fma(-w1, u0[r], u1[r]);
    const double p1 = v1[j + 1];
    bad |= !(p1 > 0.0);
    const double i1 = rsq_nr1(p1);
    const double r1 = i1 * i1;
    const double aj = ca[j];
    const double t0 = aj * r0;
    ca[j] = aj * i0;
    const double aj1 = fma(-u0[j + 1], t0, ca[j + 1]);
    const double t1 = aj1 * r1;
    ca[j + 1] = aj1 * i1;
    if (j + 2 < kCholNb) {
      ca[j + 2] = fma(-v1[j + 2], t1, fma(-u0[j + 2], t0, ca[j + 2]));
      ca[j + 3] = fma(-v1[j + 3], t1, fma(-u0[j + 3], t0, ca[j + 3]));
      if (lane < kCholNb) {
        prw[lane] = ca[j + 2];
        prw2[lane] = ca[j + 3];
      }
    }
#pragma unroll
    for (int r = j + 4; r < kCholNb; ++r) ca[r] = fma(-v1[r], t1, fma(-u0[r], t0, ca[r]));
#pragma unroll
    for (int r = j; r < kCholNb; ++r) asm volatile("" : "+v"(ca[r]));
    if (j + 2 < kCholNb) {
#pragma unroll
      for (int r = j + 2; r < kCholNb; ++r) {
        u0[r] = prw[r];
        u1[r] = prw2[r];
      }
    }
  }
  return bad;
}

// The same factorisation with the pivot rows broadcast by v_readlane (wave-uniform SGPR multipliers, no LDS
// round trip on the pivot chain), two pivots per step: rows j and j+1 are read together and every lane
// derives pivot j+1's row from them (uniform arithmetic), then applies both eliminations to its own column.
// Same arithmetic as tile_factor up to rounding (the second pivot row is formed as in tile_factor's v1).
__device__ __forceinline__ bool tile_factor_rl(const double* D, const double* Yk, const double* Id,
                                               double (&ca)[16]) {
  const int lane = opaque_lane();
  const int c = lane & 15;
  const bool isy = lane == 32;
  const double* b0 = isy ? Yk : ((lane >= 16 && lane < 32) ? Id + c : D + c);
  const int rs = isy ? 1 : kTLd;
#pragma unroll
  for (int r = 0; r < kCholNb; ++r) ca[r] = b0[r * rs];
  bool bad = false;
#pragma unroll
  for (int j = 0; j < kCholNb; j += 2) {
    double a[kCholNb], b[kCholNb];   // raw rows j and j+1 at columns >= j / >= j+1 (uniform)
#pragma unroll
    for (int r = j; r < kCholNb; ++r) a[r] = readlane_d(ca[j], r);
#pragma unroll
    for (int r = j + 1; r < kCholNb; ++r) b[r] = readlane_d(ca[j + 1], r);
    const double p0 = a[j];
    bad |= !(p0 > 0.0);
    const double i0 = rsq_nr1(p0);
    const double r0 = i0 * i0;
    const double w1 = a[j + 1] * r0;
    const double p1 = fma(-w1, a[j + 1], b[j + 1]);
    bad |= !(p1 > 0.0);
    const double i1 = rsq_nr1(p1);
    const double r1 = i1 * i1;
    const double cj = ca[j];
    const double t0 = cj * r0;
    ca[j] = cj * i0;
    const double cj1 = fma(-a[j + 1], t0, ca[j + 1]);
    const double t1 = cj1 * r1;
    ca[j + 1] = cj1 * i1;
#pragma unroll
    for (int r = j + 2; r < kCholNb; ++r) ca[r] = fma(-fma(-w1, a[r], b[r]), t1, fma(-a[r], t0, ca[r]));
  }
  return bad;
}

// The four 16-lane rows' values of x at this lane's column: g[m] = x at lane li + 16 m (gfx950 permlane swaps,
// as in sum_rows4: no LDS round trip).
__device__ __forceinline__ void col_gather4(double x, double (&g)[4]) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);   // [0]: lane l & 31, [1]: (l & 31) + 32
  auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  auto c = __builtin_amdgcn_permlane16_swap(a[0], a[0], false, false);   // [0]: bit 4 clear, [1]: set
  auto e = __builtin_amdgcn_permlane16_swap(b[0], b[0], false, false);
  auto f = __builtin_amdgcn_permlane16_swap(a[1], a[1], false, false);
  auto h = __builtin_amdgcn_permlane16_swap(b[1], b[1], false, false);
  g[0] = __hiloint2double(e[0], c[0]);
  g[1] = __hiloint2double(e[1], c[1]);
  g[2] = __hiloint2double(h[0], f[0]);
  g[3] = __hiloint2double(h[1], f[1]);
}

// The diagonal tile's factorisation in registers, in the MFMA layout it arrives in (no LDS staging, no
// broadcast per pivot): four panels of four rows.  Panel p: the 4x4 block B of rows / columns 4p..4p+3 comes
// to every lane by v_readlane and is factored wave-uniformly (B = R^T R); each lane transforms the four panel
// rows at its column by R^-T (row-wise forward substitution; the rows' values at the column gathered by
// permlane swaps) and keeps its own row's; the trailing rows then take the panel's rank-4 update as ONE
// v_mfma_f64_16x16x4f64 (A = B = the new panel register: C -= U_pan^T U_pan).  The identity takes the same row
// operations (-> Z = U^-T, one more MFMA per panel) and so does the rhs (y[li] on the lanes of column li).
// In: D (acc layout: D[q] = D[lk + 4q][li], upper triangle meaningful), ys = y[li].  Out: Zt[q] =
// Z[lk + 4q][li], ys = z[li] = (Z y)[li].  16 pivots = 4 uniform 4-pivot chains and 8 MFMAs, against 8 LDS
// broadcast rounds in tile_factor.  Returns true on a non-positive pivot.
__device__ __forceinline__ bool tile_factor_mfma(const f64x4& D, double& ys, f64x4& Zt, int li, int lk) {
  f64x4 A, E;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    A[q] = (lk + 4 * q <= li) ? D[q] : 0.0;
    E[q] = (lk + 4 * q == li) ? 1.0 : 0.0;
  }
  bool bad = false;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const double x = A[p], ex = E[p];
    // the 4x4 diagonal block (upper) and the panel's rhs, wave-uniform
    const double b00 = readlane_d(x, 4 * p), b01 = readlane_d(x, 4 * p + 1), b02 = readlane_d(x, 4 * p + 2),
                 b03 = readlane_d(x, 4 * p + 3);
    const double b11 = readlane_d(x, 16 + 4 * p + 1), b12 = readlane_d(x, 16 + 4 * p + 2),
                 b13 = readlane_d(x, 16 + 4 * p + 3);
    const double b22 = readlane_d(x, 32 + 4 * p + 2), b23 = readlane_d(x, 32 + 4 * p + 3);
    const double b33 = readlane_d(x, 48 + 4 * p + 3);
    const double yo[4] = {readlane_d(ys, 4 * p), readlane_d(ys, 4 * p + 1), readlane_d(ys, 4 * p + 2),
                          readlane_d(ys, 4 * p + 3)};
    double g[4], h[4];
    col_gather4(x, g);
    col_gather4(ex, h);
    // B = R^T R (R upper), pivots by rsq + one Newton step as in tile_factor
    bad |= !(b00 > 0.0);
    const double i0 = rsq_nr1(b00);
    const double r01 = b01 * i0, r02 = b02 * i0, r03 = b03 * i0;
    const double c11 = fma(-r01, r01, b11);
    bad |= !(c11 > 0.0);
    const double i1 = rsq_nr1(c11);
    const double r12 = fma(-r01, r02, b12) * i1, r13 = fma(-r01, r03, b13) * i1;
    const double c22 = fma(-r12, r12, fma(-r02, r02, b22));
    bad |= !(c22 > 0.0);
    const double i2 = rsq_nr1(c22);
    const double r23 = fma(-r12, r13, fma(-r02, r03, b23)) * i2;
    const double c33 = fma(-r23, r23, fma(-r13, r13, fma(-r03, r03, b33)));
    bad |= !(c33 > 0.0);
    const double i3 = rsq_nr1(c33);
    // new panel rows = R^-T (old panel rows): forward substitution
    auto fs = [&](const double (&o)[4], double (&w)[4]) {
      w[0] = o[0] * i0;
      w[1] = fma(-r01, w[0], o[1]) * i1;
      w[2] = fma(-r12, w[1], fma(-r02, w[0], o[2])) * i2;
      w[3] = fma(-r23, w[2], fma(-r13, w[1], fma(-r03, w[0], o[3]))) * i3;
    };
    double gn[4], hn[4], yn[4];
    fs(g, gn);
    fs(h, hn);
    fs(yo, yn);
    const double gl = lk == 0 ? gn[0] : (lk == 1 ? gn[1] : (lk == 2 ? gn[2] : gn[3]));
    const double xn = li >= 4 * p + lk ? gl : 0.0;   // row 4p + lk of U at column li (zero left of the diagonal)
    const double en = lk == 0 ? hn[0] : (lk == 1 ? hn[1] : (lk == 2 ? hn[2] : hn[3]));
    // rhs: the panel rows replaced, the trailing rows take the panel's column-li entries
    const double yt = fma(-gn[3], yn[3], fma(-gn[2], yn[2], fma(-gn[1], yn[1], fma(-gn[0], yn[0], ys))));
    const int dl = li - 4 * p;
    const double yp = dl == 0 ? yn[0] : (dl == 1 ? yn[1] : (dl == 2 ? yn[2] : yn[3]));
    ys = dl < 0 ? ys : (dl < 4 ? yp : yt);
    // trailing rank-4 updates (rows of earlier panels see zero panel entries; row block p is replaced)
    if (p < 3) A = __builtin_amdgcn_mfma_f64_16x16x4f64(-xn, xn, A, 0, 0, 0);
    E = __builtin_amdgcn_mfma_f64_16x16x4f64(-xn, en, E, 0, 0, 0);
    A[p] = xn;
    E[p] = en;
  }
  Zt = E;
  return bad;
}

// The owner of the next diagonal, register factorisation (kLa bit 3): D -> Z_K, z_K posted to the LDS ring.
__device__ __forceinline__ bool tile_diag_mfma(const f64x4& D, double ypart, TileShared& sh, int K, int li,
                                               int lk) {
  double ys = sum_rows4(ypart);
  f64x4 Zt;
  const bool bad = tile_factor_mfma(D, ys, Zt, li, lk);
  double* Zs = sh.Zs[K & 3];
#pragma unroll
  for (int q = 0; q < 4; ++q) Zs[(lk + 4 * q) * kTLd + li] = Zt[q];
  if (lk == 0) sh.zK[K & 3][li] = ys;
  return bad;
}

// The owner of the next diagonal: D (acc layout) and its rhs partials -> Z, z and Z^T z of tile row K.
template <bool kRl = false>
__device__ __forceinline__ bool tile_diag(const f64x4& D, double ypart, TileShared& sh, double* zp, int K,
                                          int lane, int li, int lk) {
#pragma unroll
  for (int q = 0; q < 4; ++q) sh.Dw[(lk + 4 * q) * kTLd + li] = (lk + 4 * q <= li) ? D[q] : 0.0;
  const double ys = sum_rows4(ypart);
  if (lk == 0) sh.Yw[li] = ys;
  double ca[kCholNb];
  const bool bad = kRl ? tile_factor_rl(sh.Dw, sh.Yw, sh.Id, ca) : tile_factor(sh.Dw, sh.Yw, sh.Id, sh.prw, ca);
  double* Zs = sh.Zs[K & 3];
  double* zk = sh.zK[K & 3];
  if (lane >= 16 && lane < 32) {
#pragma unroll
    for (int r = 0; r < kCholNb; ++r) Zs[r * kTLd + (lane - 16)] = ca[r];
  }
  if (lane == 32) {
#pragma unroll
    for (int r = 0; r < kCholNb; ++r) zk[r] = ca[r];
  }
  return bad;
}

// z'_K = Z_K^T z_K for the back substitution, from the posted Z_K and z_K (LDS ring slot K & 3): formed by
// the owner one phase later (its late phase), off the pivot chain.
// zg (bordered mode): Z_K row-major into slot 0 of W row K (W tiles start at slot 1), for k_chol_border.
__device__ __forceinline__ void tile_zp(const TileShared& sh, double* zp, int K, int lane, double* zg = nullptr) {
  if (lane < 16) {
    const double* Zs = sh.Zs[K & 3];
    const double* zk = sh.zK[K & 3];
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < kCholNb; ++r) s = fma(Zs[r * kTLd + lane], zk[r], s);
    zp[16 * K + lane] = s;
  }
  if (zg) {
    const double* Zs = sh.Zs[K & 3];
    double* dst = zg + (size_t)K * kTB * 256;
#pragma unroll
    for (int e = lane; e < 256; e += 64) dst[e] = Zs[(e >> 4) * kTLd + (e & 15)];
  }
}

// Dinv mode (flags bit 5): D_K^-1 = Z_K^T Z_K (one MFMA chain from the posted Z_K) and z'_K, posted for the
// phase's other waves by the wave that factored D_K (in its late step), released by dflag = K.
__device__ __forceinline__ void tile_dinv_post(TileShared& sh, double* zp, int K, int lane, int li, int lk,
                                               double* zg = nullptr) {
  const double* Zs = sh.Zs[K & 3];
  double zt[4];
  f64x4 zb;
#pragma unroll
  for (int s = 0; s < 4; ++s) zb[s] = zt[s] = Zs[(4 * s + lk) * kTLd + li];
  const f64x4 zero = {0.0, 0.0, 0.0, 0.0};
  const f64x4 Dv = mfma_f64_k16(zt, zb, zero);   // (Z^T Z)[lk + 4q][li]
#pragma unroll
  for (int q = 0; q < 4; ++q) sh.Dv[(lk + 4 * q) * kTLd + li] = Dv[q];
  tile_zp(sh, zp, K, lane, zg);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) __hip_atomic_store(&sh.dflag, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Diagnostic stamps (SG_STAMP=1): lane 0 of every wave accumulates s_memtime deltas per phase; waves 0 and 1
// report (tools/tile_stamps.py).
#define SG_TSTAMP(slot)                                                                  \
  if (kStamp && lane == 0) {                                                             \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                       \
    tacc[slot] += now_ - tlast;                                                          \
    tlast = now_;                                                                        \
  }
// Per-phase absolute times (SG_STAMP=1 builds; tools/phase_trace.py): d.stamps[64 + (wg 128 + K) 16 + slot],
// slots 0-7 the waves' barrier arrivals, 8-12 the owner's chain (start, after (0), TRSM, D update, factor).
constexpr int kTraceK = 128;
constexpr int kUlStamp = 64 + 2 * kTraceK * 16;   // k_update_lin's stamps (after the phase trace)
#define SG_PTRACE(K, slot)                                                                  \
  if (kStamp && lane == 0 && (K) < kTraceK)                                                \
    d.stamps[64 + ((size_t)blockIdx.x * kTraceK + (K)) * 16 + (slot)] = __builtin_amdgcn_s_memtime();

// W_KJ = Z_K^T U_KJ (= U_KK^-1 U_KJ) of one row-K tile, and its store to global memory for the back
// substitution (kept apart so that loads issued in between do not reuse the stores' data registers, which
// would wait for the stores).
__device__ __forceinline__ f64x4 tile_w(const f64x4& U, const double* Zs, int li, int lk) {
  const f64x4 zero = {0.0, 0.0, 0.0, 0.0};
  double zt[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) zt[s] = Zs[(4 * s + lk) * kTLd + li];
  return mfma_f64_k16(zt, U, zero);
}
__device__ __forceinline__ void tile_w_store(const f64x4& Wt, double* __restrict__ Wg, int K, int J, int lane) {
  double* wg = Wg + ((size_t)K * kTB + (J - K)) * 256 + lane;
#pragma unroll
  for (int q = 0; q < 4; ++q) wg[q * 64] = Wt[q];
}

// The accumulator slots rotate with the phase: in phase K, slot s of a wave's column J holds tile row
// I = J - ((J - (s + K - 1)) & 7) — row K-1 in slot 0, row K in slot 1, the next diagonal in slot 2, row
// K-1+d in slot d — and every wave rotates its slots by one between phases (register moves, off the
// critical path).  So one phase body serves every tile row and the kernel's code stays inside the
// instruction cache (a phase body instantiated per K & 7 made the kernel 150 KB, streamed through a 64 KB
// cache every eight phases).
__device__ __forceinline__ void tile_rotate(f64x4 (&acc)[kTB]) {
  const f64x4 t = acc[0];
#pragma unroll
  for (int u = 0; u < kTB - 1; ++u) acc[u] = acc[u + 1];
  acc[kTB - 1] = t;
}

// Column J of S into the slots of phase K (slot s: row J - ((J - (s + K - 1)) & 7)).
__device__ __forceinline__ void tile_col_load(f64x4 (&acc)[kTB], double& ypart, const Dev& d, int J, int K,
                                              int li, int lk, const TileSrc& ts) {
#pragma unroll
  for (int u = 0; u < kTB; ++u) acc[u] = tile_load(d.S, J - ((J - (u + K - 1)) & 7), J, li, lk, ts);
  const int gj = 16 * J + li, ld = ts.ld;
  const int sj = ts.rev ? ts.np - 1 - gj : gj;
  ypart = d.S[(lk == 0 && sj < ts.nb && J < ts.sep) ? ld * ld + sj : ld * ld + ld];
}

// One phase (tile row K) of a wave.  `late`: this wave owned the diagonal of the previous phase and still
// owes that phase's W tile and its column reload (it has no other work in this phase).
// Owner look-ahead (flags bit 3): the next phase's owner (column K+2) applies row K's update to its row-(K+1)
// tile in phase K — U_{K,K+1} is posted by this phase's owner right after its TRSM (an LDS flag, no barrier)
// — so that update (four MFMAs) leaves the next phase's critical chain (TRSM -> D update -> factor).  The
// row-(K+1) tile exists iff K + 2 < tend[K] (the band is contiguous), the same condition both phases test.
constexpr int kLaSpinMax = 1 << 20;
__device__ __forceinline__ bool la_done(int la, const int* tend, int Kp) {   // look-ahead ran in phase Kp
  return (la & 1) && Kp >= 0 && Kp + 2 < tend[Kp];
}

template <bool kStamp>
__device__ __forceinline__ void tile_phase(f64x4 (&acc)[kTB], double& ypart, int& J, bool& late, bool& bad,
                                           bool& tmo, int la, TileShared& sh, const Dev& d,
                                           double* __restrict__ Wg, double* zp, const int* tend, int K, int NT,
                                           int lane, int li, int lk, const TileSrc& ts, double* zg,
                                           unsigned long long (&tacc)[16], unsigned long long& tlast) {
  if (late) {
    // the previous phase's owner (column J = K): its row K-1 tile (slot 0) -> W, then column J + 8, which
    // row K + 1 touches first
    const bool hasw = J < tend[K - 1];
    f64x4 Wt = {0.0, 0.0, 0.0, 0.0};
    if (hasw) Wt = tile_w(acc[0], sh.Zs[(K - 1) & 3], li, lk);
    const int Jw = J;
    if (la & 4) tile_dinv_post(sh, zp, K, lane, li, lk, zg);   // D_K^-1 and z'_K for the phase's other waves first
    J += kTB;
    tile_col_load(acc, ypart, d, J, K, li, lk, ts);
    if (hasw) tile_w_store(Wt, Wg, K - 1, Jw, lane);
    if (!(la & 4)) tile_zp(sh, zp, K, lane, zg);   // the diagonal this wave factored last phase
    late = false;
    SG_TSTAMP(13)
    return;
  }
  if (J == K + 1) SG_PTRACE(K, 8)
  // (0) trailing update by row K-1 (the owner's diagonal tile, dd = 2, already took it last phase; with the
  // look-ahead its row-K tile, dd = 1, too)
  if (K >= 1 && J < tend[K - 1]) {
    const double* Ub = sh.Ur[(K - 1) & 1][0];
    const bool own_la = J == K + 1 && la_done(la, tend, K - 1);
#pragma unroll
    for (int dd = 1; dd < kTB; ++dd) {
      if (K - 1 + dd <= J && !(dd == 2 && J == K + 1) && !(dd == 1 && own_la)) {
        double a[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = -Ub[(dd - 1) * 256 + s * 64 + lane];
        acc[dd] = mfma_f64_k16(a, acc[0], acc[dd]);
      }
    }
  }
  SG_TSTAMP(8)
  if (J == K + 1) SG_PTRACE(K, 9)
  // (1) TRSM of row K's tile
  const int te = tend[K];
  const bool act = J < te;
  const double* Zs = sh.Zs[K & 3];
  if ((la & 4) && act && J != K + 1) {
    // Dinv mode, a column off the critical chain: no TRSM.  Its raw row-K tile A_KJ goes to the exchange
    // ring (the trailing updates become A_IJ -= A_KI^T W_KJ), W_KJ = D_K^-1 A_KJ (= U_KK^-1 U_KJ) is both the
    // back-substitution tile and this column's operand for the next phase's update, and the rhs term is
    // A_KJ^T z'_K (= U_KJ^T z_K).
    const f64x4 A = acc[1];
    double* ur = sh.Ur[K & 1][J - K - 1];
#pragma unroll
    for (int q = 0; q < 4; ++q) ur[q * 64 + lane] = A[q];
    int spin = 0;
    while (__hip_atomic_load(&sh.dflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < K && ++spin < kLaSpinMax)
      __builtin_amdgcn_s_sleep(0);
    tmo |= spin >= kLaSpinMax;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    double da[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) da[s] = sh.Dv[li * kTLd + 4 * s + lk];
    const f64x4 zero = {0.0, 0.0, 0.0, 0.0};
    const f64x4 W = mfma_f64_k16(da, A, zero);
#pragma unroll
    for (int q = 0; q < 4; ++q) ypart = fma(-A[q], zp[16 * K + lk + 4 * q], ypart);
    tile_w_store(W, Wg, K, J, lane);
    acc[1] = W;
    if (J == K + 2) {
      double a[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) a[s] = -A[s];
      acc[3] = mfma_f64_k16(a, W, acc[3]);   // D_{K+2} -= A_{K,K+2}^T W_{K,K+2}
      if (la_done(la, tend, K)) {
        int spin2 = 0;
        while (__hip_atomic_load(&sh.uflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < K &&
               ++spin2 < kLaSpinMax)
          __builtin_amdgcn_s_sleep(0);
        tmo |= spin2 >= kLaSpinMax;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const double* A1 = sh.Ur[K & 1][0];   // the owner's raw A_{K,K+1}
        double b1[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) b1[s] = -A1[s * 64 + lane];
        acc[2] = mfma_f64_k16(b1, W, acc[2]);   // A_{K+1,K+2} -= A_{K,K+1}^T W_{K,K+2}
      }
    }
    SG_TSTAMP(9)
    return;
  }
  if ((la & 4) && act && J == K + 1) {
    // Dinv mode, the owner: its raw row-K tile to the ring first (the next owner's look-ahead operand)
    double* ur = sh.Ur[K & 1][0];
#pragma unroll
    for (int q = 0; q < 4; ++q) ur[q * 64 + lane] = acc[1][q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(&sh.uflag, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (act) {
    const f64x4 zero = {0.0, 0.0, 0.0, 0.0};
    double za[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) za[s] = Zs[li * kTLd + 4 * s + lk];
    const f64x4 U = mfma_f64_k16(za, acc[1], zero);
    acc[1] = U;
    double* ur = sh.Ur[K & 1][J - K - 1];
    if (!(la & 4)) {
#pragma unroll
      for (int q = 0; q < 4; ++q) ur[q * 64 + lane] = U[q];
    }
    if ((la & 1) && !(la & 4) && J == K + 1) {
      // the owner: U_{K,K+1} is the next owner's look-ahead operand (in-order LDS: data, then the flag)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&sh.uflag, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if ((la & 16) && !(la & 4)) {
      // dataflow mode: this column's U_{K,J} is in the ring (counted; the next phase waits for the whole row)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_fetch_add(&sh.uposted, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const double* zk = sh.zK[K & 3];
#pragma unroll
    for (int q = 0; q < 4; ++q) ypart = fma(-U[q], zk[lk + 4 * q], ypart);
    if (J == K + 2 && !(la & 4)) {
      // next phase's owner: its diagonal tile's update by row K uses only its own U_{K,J}; apply it now,
      // off next phase's critical chain (slot 3 = row K + 2)
      double a[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) a[s] = -U[s];
      acc[3] = mfma_f64_k16(a, U, acc[3]);
      if (la_done(la, tend, K)) {
        // look-ahead: the row-(K+1) tile (slot 2) takes row K's update now, U_{K,K+1} from the owner
        int spin = 0;
        while (__hip_atomic_load(&sh.uflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < K &&
               ++spin < kLaSpinMax)
          __builtin_amdgcn_s_sleep(0);
        tmo |= spin >= kLaSpinMax;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const double* U1 = sh.Ur[K & 1][0];
        double b1[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) b1[s] = -U1[s * 64 + lane];
        acc[2] = mfma_f64_k16(b1, U, acc[2]);
      }
    }
  }
  SG_TSTAMP(9)
  if (J == K + 1) {
    SG_PTRACE(K, 10)
    // (2) the next diagonal: apply row K, factor, post; its W tile and the reload follow next phase
    if (act) {
      double a[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) a[s] = -acc[1][s];
      acc[2] = mfma_f64_k16(a, acc[1], acc[2]);
    }
    SG_TSTAMP(10)
    SG_PTRACE(K, 11)
    if (K + 1 < NT) {
      bad |= (la & 8) ? tile_diag_mfma(acc[2], ypart, sh, K + 1, li, lk)
             : (la & 2) ? tile_diag<true>(acc[2], ypart, sh, zp, K + 1, lane, li, lk)
                        : tile_diag<false>(acc[2], ypart, sh, zp, K + 1, lane, li, lk);
      if (la & 16) {   // dataflow mode: Z_{K+1}, z_{K+1} posted
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&sh.zflag, K + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    SG_PTRACE(K, 12)
    late = true;
    SG_TSTAMP(11)
  } else if (act) {
    // (3) back-substitution tile
    tile_w_store(tile_w(acc[1], Zs, li, lk), Wg, K, J, lane);
    SG_TSTAMP(12)
  }
}

// The bottom half's step after its last factored row ND-1 (slots of phase ND): the previous owner's W tile,
// and every other wave's update of its separator column by row ND-1 ((0) of a phase, nothing else).
__device__ __forceinline__ void tile_final(f64x4 (&acc)[kTB], int J, bool& late, int la, TileShared& sh,
                                           double* __restrict__ Wg, const int* tend, int K, int lane, int li,
                                           int lk) {
  if (late) {
    if (J < tend[K - 1]) tile_w_store(tile_w(acc[0], sh.Zs[(K - 1) & 3], li, lk), Wg, K - 1, J, lane);
    late = false;
    return;
  }
  if (J < tend[K - 1]) {
    const double* Ub = sh.Ur[(K - 1) & 1][0];
    const bool own_la = J == K + 1 && la_done(la, tend, K - 1);
#pragma unroll
    for (int dd = 1; dd < kTB; ++dd) {
      // (the diagonal of column K+1: applied early; its row-K tile too under the look-ahead)
      if (K - 1 + dd <= J && !(dd == 2 && J == K + 1) && !(dd == 1 && own_la)) {
        double a[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = -Ub[(dd - 1) * 256 + s * 64 + lane];
        acc[dd] = mfma_f64_k16(a, acc[0], acc[dd]);
      }
    }
  }
}

// Separator hand-off.  The bottom half writes its contribution to the separator tiles (its columns
// ND..ND+6, rows >= ND) mapped back to S's order — reversed tile (I', J') element (a, b) is tile
// (NT-1-J', NT-1-I') element (15-b, 15-a) — in the top half's accumulator layout, and its rhs partials
// summed over the lane rows.
__device__ __forceinline__ void sep_write(const f64x4 (&acc)[kTB], double ypart, int J, int ND, int NT, int m,
                                          double* __restrict__ sepb, double* __restrict__ sepy, int li, int lk) {
  if (J < ND || J >= ND + 7) return;
  const double ys = sum_rows4(ypart);
  const int Io = NT - 1 - J;
#pragma unroll
  for (int u = 0; u < kTB; ++u) {
    const int I = J - ((J - (u + ND - 1)) & 7);   // slots of phase ND
    if (I >= ND) {
      double* dst = sepb + ((Io - m) * 7 + (NT - 1 - I - m)) * 256;
      const int C0 = 15 - li;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int Rd = C0, Cd = 15 - (lk + 4 * q);   // source (a, b) = (lk + 4q, li) -> (15 - b, 15 - a)
        dst[(Rd >> 2) * 64 + Cd + 16 * (Rd & 3)] = acc[u][q];
      }
    }
  }
  if (lk == 0) sepy[(Io - m) * 16 + 15 - li] = ys;
}

// The top half adds the bottom half's separator contribution to the separator columns it holds (before
// the first separator diagonal is factored).
__device__ __forceinline__ void sep_merge(f64x4 (&acc)[kTB], double& ypart, int J, int m,
                                          const double* __restrict__ sepb, const double* __restrict__ sepy,
                                          int lane, int li, int lk) {
  if (J < m || J >= m + 7) return;
#pragma unroll
  for (int u = 0; u < kTB; ++u) {
    const int I = J - ((J - (u + m - 2)) & 7);   // slots of phase m - 1
    if (I >= m) {
      const double* src = sepb + ((I - m) * 7 + (J - m)) * 256 + lane;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[u][q] += src[q * 64];
    }
  }
  if (lk == 0) ypart += sepy[(J - m) * 16 + li];
}

// Back substitution of tile rows Khi .. Klo in one wave:  x_K = z'_K - sum_{d=1..7} W_{K,K+d} x_{K+d}, with no
// LDS round trip on the row-to-row chain.  Lane (li, lk) holds rows lk + 4q, column li of each W tile (acc
// layout) and x_{K+d}[li] in registers (xw[d-1]; zero past the last row, and W tiles outside the band are
// zero), so the d >= 2 terms are formed before x_{K+1} is known.  The 16-lane row sums run as a DPP butterfly
// (quad xor 1, quad xor 2, half-row mirror, row mirror: bitwise the same sum in every lane), and one shuffle
// moves x_K[li] (row li & 3, register li >> 2) to every lane.  W rows are prefetched two rows ahead (two
// register buffers, the loop unrolled by two); z' is read one row ahead.  kRev: the rows are the bottom
// half's reversed order, x_K[li] is stored at S-order index 16 (NT-1-K) + 15 - li.
template <bool kRev>
__device__ __forceinline__ void bs_chain(const double* __restrict__ Wb, const double* zsrc, double* xs, int Khi,
                                         int Klo, double (&xw)[kTB - 1], int NT, int lane, int li, int lk) {
  auto wload = [&](double (&w)[kTB - 1][4], int K) {
    const double* src = Wb + (size_t)(K >= 0 ? K : 0) * kTB * 256 + lane;
#pragma unroll
    for (int dd = 1; dd < kTB; ++dd)
#pragma unroll
      for (int q = 0; q < 4; ++q) w[dd - 1][q] = src[dd * 256 + q * 64];
  };
  const int srcl = 16 * (li & 3) + li;   // the lane holding x_K[li] after the row sums
  unsigned qbits = 1u << (li >> 2);
  asm volatile("" : "+v"(qbits));
  auto bs_row = [&](int K, double (&w)[kTB - 1][4], const double (&zk)[4]) {
    double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int dd = kTB - 1; dd >= 1; --dd)
#pragma unroll
      for (int q = 0; q < 4; ++q) p[q] = fma(w[dd - 1][q], xw[dd - 1], p[q]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double v = p[q];
      v += dpp_d<0xB1>(v);
      v += dpp_d<0x4E>(v);
      v += dpp_d<0x141>(v);
      v += dpp_d<0x140>(v);
      p[q] = zk[q] - v;   // x_K[lk + 4q], the same bits in every lane of the row
    }
    // register p[li >> 2] by opaque bit masks (a lane-dependent ?: chain compiles to divergent branches)
    unsigned long long mb = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int msk;
      asm volatile("v_bfe_i32 %0, %1, %2, 1" : "=v"(msk) : "v"(qbits), "n"(q));
      mb |= (unsigned long long)__double_as_longlong(p[q]) & (unsigned long long)(long long)msk;
    }
    const double xk = __shfl(__longlong_as_double((long long)mb), srcl);
    if (kRev)
      xs[16 * (NT - 1 - K) + 15 - li] = xk;
    else
      xs[16 * K + li] = xk;   // the same bits from every row of lanes
#pragma unroll
    for (int dd = kTB - 2; dd >= 1; --dd) xw[dd] = xw[dd - 1];
    xw[0] = xk;
    wload(w, K - 2);   // this buffer's next row
  };
  double wA[kTB - 1][4], wB[kTB - 1][4], zA[4], zB[4];
  wload(wA, Khi);
  wload(wB, Khi - 1);
#pragma unroll
  for (int q = 0; q < 4; ++q) zA[q] = zsrc[16 * Khi + lk + 4 * q];
  int K = Khi;
  for (; K >= Klo + 1; K -= 2) {
#pragma unroll
    for (int q = 0; q < 4; ++q) zB[q] = zsrc[16 * (K - 1) + lk + 4 * q];
    bs_row(K, wA, zA);
#pragma unroll
    for (int q = 0; q < 4; ++q) zA[q] = zsrc[16 * (K >= 2 ? K - 2 : 0) + lk + 4 * q];
    bs_row(K - 1, wB, zB);
  }
  if (K == Klo) bs_row(K, wA, zA);
}

// The same chain on two waves: wave `par` takes rows Khi - par, Khi - par - 2, ..., so each wave has two
// rows' time to bring in its next W rows (its register buffers hold rows 2 and 4 ahead of the chain); the
// other wave's newest x arrives through LDS behind a per-row flag (`done[K]`: set after x_K is written; the
// LDS accesses of one wave execute in order).  xw: x_{Khi+1 .. Khi+7} (zero past the system).  The flag wait
// is bounded; a time-out sets `tmo` (counted in kCTimeout: the solve then ends with SG_DEVICE_TIMEOUT).
template <bool kRev>
__device__ __forceinline__ void bs_chain2(const double* __restrict__ Wb, const double* zsrc, double* xs,
                                          int* done, int Khi, int Klo, double (&xw)[kTB - 1], int NT, int par,
                                          int lane, int li, int lk, bool& tmo) {
  auto xat = [&](int K) -> double& { return kRev ? xs[16 * (NT - 1 - K) + 15 - li] : xs[16 * K + li]; };
  auto wload = [&](double (&w)[kTB - 1][4], int K) {
    const double* src = Wb + (size_t)(K >= 0 ? K : 0) * kTB * 256 + lane;
#pragma unroll
    for (int dd = 1; dd < kTB; ++dd)
#pragma unroll
      for (int q = 0; q < 4; ++q) w[dd - 1][q] = src[dd * 256 + q * 64];
  };
  const int srcl = 16 * (li & 3) + li;
  unsigned qbits = 1u << (li >> 2);
  asm volatile("" : "+v"(qbits));
  double xown = 0.0;   // this wave's previous result (x_{K+2} at row K)
  auto wait_row = [&](int K) {   // x_K of the other wave
    int spin = 0;
    while (__hip_atomic_load(done + K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0 && ++spin < (1 << 20))
      __builtin_amdgcn_s_sleep(0);
    tmo |= spin >= (1 << 20);
    asm volatile("" ::: "memory");
  };
  auto bs_row = [&](int K, double (&w)[kTB - 1][4], const double (&zk)[4], bool first) {
    // window x_{K+1 .. K+7}
    if (K + 1 <= Khi) {
      wait_row(K + 1);
      const double xo = xat(K + 1);
      if (first) {   // par 1's first row: x_{Khi} ahead of the initial window
#pragma unroll
        for (int dd = kTB - 2; dd >= 1; --dd) xw[dd] = xw[dd - 1];
        xw[0] = xo;
      } else {       // two new rows: the other wave's x_{K+1}, this wave's x_{K+2}
#pragma unroll
        for (int dd = kTB - 2; dd >= 2; --dd) xw[dd] = xw[dd - 2];
        xw[1] = xown;
        xw[0] = xo;
      }
    }
    double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int dd = kTB - 1; dd >= 1; --dd)
#pragma unroll
      for (int q = 0; q < 4; ++q) p[q] = fma(w[dd - 1][q], xw[dd - 1], p[q]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double v = p[q];
      v += dpp_d<0xB1>(v);
      v += dpp_d<0x4E>(v);
      v += dpp_d<0x141>(v);
      v += dpp_d<0x140>(v);
      p[q] = zk[q] - v;
    }
    unsigned long long mb = 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int msk;
      asm volatile("v_bfe_i32 %0, %1, %2, 1" : "=v"(msk) : "v"(qbits), "n"(q));
      mb |= (unsigned long long)__double_as_longlong(p[q]) & (unsigned long long)(long long)msk;
    }
    const double xk = __shfl(__longlong_as_double((long long)mb), srcl);
    xat(K) = xk;
    asm volatile("" ::: "memory");
    if (lane == 0) __hip_atomic_store(done + K, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    xown = xk;
    wload(w, K - 4);   // this buffer's next row (two of this wave's rows ahead)
  };
  const int K0 = Khi - par;
  if (K0 < Klo) return;
  double wA[kTB - 1][4], wB[kTB - 1][4], zA[4], zB[4];
  wload(wA, K0);
  wload(wB, K0 - 2);
#pragma unroll
  for (int q = 0; q < 4; ++q) zA[q] = zsrc[16 * K0 + lk + 4 * q];
  // (par 0's first row, K = Khi, keeps the initial window: bs_row skips the update when K + 1 > Khi)
  int K = K0;
  bool first = true;
  for (; K >= Klo + 2; K -= 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) zB[q] = zsrc[16 * (K - 2) + lk + 4 * q];
    bs_row(K, wA, zA, first);
    first = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) zA[q] = zsrc[16 * (K >= 4 ? K - 4 : 0) + lk + 4 * q];
    bs_row(K - 2, wB, zB, false);
  }
  if (K >= Klo) bs_row(K, wA, zA, first);
}

// Dissected band (nd > 0: two workgroups).  With m = NT - nd - 7, the tile rows split into the top part
// A = [0, m), the separator [m, m+7) and the bottom part B = [m+7, NT).  The band is at most 8 tiles wide,
// so A and B never couple: eliminating A, then B, then the separator is an exact Cholesky of S in that
// order (nested dissection), and A and B are factored at the same time.
//   * blockIdx 0 (top) runs the phases of rows 0 .. m+6 of S (band ends clamped to the separator); at
//     phase m-1 each wave waits for the bottom half and adds its separator contribution, then factors the
//     separator rows as usual.
//   * blockIdx 1 (bottom) runs the phases of B in reversed order (P S P: rows NT-1 .. m+7 of S, then the
//     separator as its trailing columns, started at zero), writes the separator contribution, its z' and
//     W tiles, and signals with a release counter.
//   * Back substitution (top workgroup): the separator rows, then A (wave 0) and B (wave 1, reversed W
//     tiles) side by side.
// The chain drops from NT tile rows to m + 7 (C2: 18 -> 13, C5: 75 -> 42).  The wait is bounded: on a
// time-out the launch reports it (kCTimeout) and the LM decision ends the solve with SG_DEVICE_TIMEOUT
// instead of hanging or silently rejecting the step.
//   flags bit 2 (SG_CHOL_FORCE_TIMEOUT, tests only): the bottom workgroup sleeps ~2 ms before its work and
//   the top one polls at most 256 times, so the time-out path runs deterministically.
constexpr int kSepSpinMax = 1 << 22;
constexpr int kSplitMinNT = 13;
template <bool kStamp, int kLa>
__global__ __launch_bounds__(kTileThreads) void k_chol_tiles(Dev d, const int32_t* panel_jend,
                                                             double* __restrict__ Wg, int32_t* tflag, int nd,
                                                             int flags) {
  const bool simdmap = (flags & 1) != 0;   // bit 0: columns J, J+1 on one SIMD; bit 1: LDS-staged candidates
  const LmState* st = d.st;
  unsigned long long tlast = kStamp ? __builtin_amdgcn_s_memtime() : 0ull, tacc[16] = {};
  __shared__ TileShared sh;
  extern __shared__ double tdyn[];
  // flags bit 3: the frame part of a system bordered by free intrinsics (order kc0 in S of pitch n): factor it,
  // keep each Z_K (slot 0 of its W row) and x_f0 = S_ff^-1 r_f for k_chol_border, which finishes the solve
  const bool border = (flags & 8) != 0;
  const int n = border ? d.kc0 : d.n, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lk = lane >> 4;
  const int NT = (n + 15) >> 4;
  const bool bottom = nd > 0 && blockIdx.x == 1;
  const int m = nd > 0 ? NT - nd - 7 : NT;   // first separator tile row (S order)
  const int NTf = nd > 0 ? (bottom ? nd : m + 7) : NT;   // tile rows this workgroup factors
  double* Wb = bottom ? Wg + (size_t)NT * kTB * 256 : Wg;
  double* zpg = Wg + (size_t)2 * NT * kTB * 256;   // [16 nd] the bottom half's z'
  double* sepb = zpg + 16 * NT;                     // [49][256] separator contribution
  double* sepy = sepb + 49 * 256;                   // [7][16]   its rhs
  const TileSrc ts{bottom ? 1 : 0, 16 * NT, bottom ? nd : (1 << 28), n, d.n};
  double* zg = border ? Wb : nullptr;
  double* xs = tdyn;              // [16 NT] back-substitution solution
  double* zp = tdyn + 16 * NT;    // [16 NT] Z_K^T z_K
  int* tend = reinterpret_cast<int*>(tdyn + 32 * NT);   // [NT] band end (tiles, exclusive) per tile row
  int* rdone = tend + NT;                                 // [NT] back substitution: row K's x is in xs
  int* rdone_b = rdone + NT;                              // [NT] the same for the bottom's reversed rows
  for (int k = tid; k < 2 * NT; k += kTileThreads) rdone[k] = 0;
  // candidate-pass operands (staged during the back substitution) after the band ends
  const bool cand_lds = (flags & 2) != 0;
  CandLds cl;
  cl.carve(tdyn + 32 * NT + (3 * NT + 1) / 2, d.F, d.D, n);
  // hand-off counter: the bottom half has finished this launch once tflag[0] exceeds the top half's count
  const int epoch = (nd > 0 && !bottom) ? tflag[1] : 0;
  if (tid == 0) {
    sh.fail = 0;
    sh.tmo = 0;
    sh.uflag = -1;
    sh.dflag = -1;
    sh.uposted = 0;
    sh.zflag = 0;   // Z_0 is posted before the first barrier
  }
  // kLa bit 0: owner look-ahead; bit 1: readlane factorisation; bit 2: Dinv mode (off-chain columns skip the
  // TRSM).  A template parameter, not a flag: each variant is its own kernel, so the default one carries none
  // of the others' code (with all three as run-time branches the kernel grew to 93 KB, past the 64 KB
  // instruction cache, and the C2 factorisation slowed from 69 to 77 us)
  constexpr int la = kLa;
  bool bad = false, tmo = false;
  const int spin_max = (flags & 4) ? 256 : kSepSpinMax;
  if (bottom && (flags & 4))
    for (int i = 0; i < 640; ++i) __builtin_amdgcn_s_sleep(127);
  // Columns J and J+1 (mod 8) on one SIMD: the owner of phase K (column K+1) then shares its SIMD with the
  // late wave of column K (one W tile, a reload) or with column K+2 (its first few tiles), not with a
  // column four ahead and its full band of trailing MFMAs.  SIMD ids from HW_ID; any other placement than
  // two waves per SIMD keeps column = wave.
  if (lane == 0) sh.simd[wave] = __builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);   // HW_ID.SIMD_ID
  for (int i = tid; i < 16 * kTLd; i += kTileThreads) sh.Id[i] = (i / kTLd == i % kTLd) ? 1.0 : 0.0;
  __syncthreads();
  int col = wave;
  if (simdmap) {
    const int my = sh.simd[wave];
    int cnt[4] = {0, 0, 0, 0}, rank = 0;
#pragma unroll
    for (int w = 0; w < kTB; ++w) {
      const int sw = sh.simd[w] & 3;
      cnt[sw] += 1;
      if (w < wave && sw == my) rank += 1;
    }
    if (cnt[0] == 2 && cnt[1] == 2 && cnt[2] == 2 && cnt[3] == 2) col = 2 * my + rank;
  }
  {
    f64x4 acc[kTB];
    double ypart = 0.0;
    int J = col;
    bool late = false;
    // the first column's loads go out before the LmState read returns (a finished solve exits after them)
    f64x4 D0;
    double y0 = 0.0;
    if (J == 0) {
      // D_0 has no updates: load it and column 8 together, then factor D_0 while column 8 arrives
      D0 = tile_load(d.S, 0, 0, li, lk, ts);
      const int sj0 = ts.rev ? ts.np - 1 - li : li, ld = ts.ld;
      y0 = d.S[(lk == 0 && sj0 < n && 0 < ts.sep) ? ld * ld + sj0 : ld * ld + ld];
      J = kTB;
    }
    const int done = st->done;
    asm volatile("" ::: "memory");   // the LmState load goes out before column 8's (its wait then skips them)
    tile_col_load(acc, ypart, d, J, 0, li, lk, ts);   // slots of phase 0
    // band ends (read first in phase 0, after the barrier below): their loads follow the column's
    for (int k = tid; k < NT; k += kTileThreads) {
      if (!bottom) {
        tend[k] = min((panel_jend[k] + 15) >> 4, NTf);
      } else {
        // reversed row k = column c = NT-1-k of S: its band reaches back to lo(c), the first row whose band
        // covers c (band ends are non-decreasing), so the reversed row ends at NT - lo(c)
        const int c = NT - 1 - k;
        int lo = c;
        for (int i = max(0, c - kTB); i < c; ++i)
          if (((panel_jend[i] + 15) >> 4) > c) { lo = i; break; }
        tend[k] = min(NT - lo, nd + 7);
      }
    }
    if (done) return;
    if (col == 0) {
      bad |= (la & 8) ? tile_diag_mfma(D0, y0, sh, 0, li, lk)
             : (la & 2) ? tile_diag<true>(D0, y0, sh, zp, 0, lane, li, lk)
                        : tile_diag<false>(D0, y0, sh, zp, 0, lane, li, lk);
      if (la & 4)
        tile_dinv_post(sh, zp, 0, lane, li, lk, zg);
      else
        tile_zp(sh, zp, 0, lane, zg);   // (the wave's own LDS writes: visible to it in order)
    }
    else if (cand_lds)   // the seven waves that wait at the first barrier
      cand_prefetch(d, cl, st->cur, (col - 1) * 64 + lane, kTileThreads - 64);
    SG_TSTAMP(0)
    __syncthreads();
    SG_TSTAMP(1)
    // Dataflow mode (kLa bit 4): no barrier between phases.  Phase K needs row K-1's U tiles (all of them: the
    // trailing updates) and Z_K / z_K (the TRSM); each wave waits for exactly those (a monotonic count of posted
    // U tiles against the running total of row sizes, and the Z flag), so the next owner starts its TRSM the
    // moment Z_K is posted instead of at a barrier that also waits for every trailing update.  Ring safety: a
    // wave that has seen all of row K-1 posted knows every wave has finished reading row K-2 (the U ring is two
    // deep) and has passed phase K-2 (the Z ring is four deep).  Bounded waits (kCTimeout on expiry).
    int uexp = 0;
    auto df_wait = [&](int K) {
      uexp += max(0, tend[K - 1] - K);   // row K-1's U tiles: columns K .. tend[K-1]-1
      int spin = 0;
      while ((__hip_atomic_load(&sh.uposted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < uexp ||
              __hip_atomic_load(&sh.zflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < K) &&
             ++spin < kLaSpinMax)
        __builtin_amdgcn_s_sleep(0);
      tmo |= spin >= kLaSpinMax;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
#pragma nounroll
    for (int K = 0; K < NTf; ++K) {
      if ((la & 16) && K >= 1) df_wait(K);
      if (nd > 0 && !bottom && K == m - 1) {
        // relaxed polls, one acquire (an acquiring poll would invalidate the cache on every round)
        int spin = 0;
        while (__hip_atomic_load(tflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= epoch &&
               ++spin < spin_max)
          __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        tmo |= spin >= spin_max;
        sep_merge(acc, ypart, J, m, sepb, sepy, lane, li, lk);
      }
      tile_phase<kStamp>(acc, ypart, J, late, bad, tmo, la, sh, d, Wb, zp, tend, K, NTf, lane, li, lk, ts, zg,
                         tacc, tlast);
      SG_TSTAMP(2)
      // the owner of the next diagonal (now late) is on the critical path until the barrier: it rotates after
      if (!late) tile_rotate(acc);
      SG_PTRACE(K, wave)
      if (!(la & 16)) lds_barrier();
      if (late) tile_rotate(acc);
      SG_TSTAMP(3)
    }
    if (bottom) {
      // row nd-1's updates of the separator columns (slots of phase nd), then the hand-off
      if (la & 16) {   // row nd-1 complete (no Z_nd: the bottom does not factor the separator)
        uexp += max(0, tend[nd - 1] - nd);
        int spin = 0;
        while (__hip_atomic_load(&sh.uposted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < uexp &&
               ++spin < kLaSpinMax)
          __builtin_amdgcn_s_sleep(0);
        tmo |= spin >= kLaSpinMax;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      }
      tile_final(acc, J, late, la, sh, Wb, tend, nd, lane, li, lk);
      sep_write(acc, ypart, J, nd, NT, m, sepb, sepy, li, lk);
    }
  }
  if (bottom) {
    if (bad && lane == 0) sh.fail = 1;
    __syncthreads();   // every owner's z' in LDS
    for (int i = tid; i < 16 * nd; i += kTileThreads) zpg[i] = zp[i];
    if (tid == 0) zpg[16 * nd] = sh.fail ? 1.0 : 0.0;   // failure marker (slot past z': read by the top half)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // every wave's hand-off stores, then one signal
    __syncthreads();
    if (tid == 0) {
      const int c = tflag[0];
      __hip_atomic_store(tflag, c + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (nd > 0 && zpg[16 * nd] != 0.0) bad = true;
  if (bad && lane == 0) sh.fail = 1;
  __syncthreads();   // W tiles (global) and z' visible to every wave
  SG_TSTAMP(4)
  const int cur = st->cur;
  {
    double xw[kTB - 1];
#pragma unroll
    for (int dd = 0; dd < kTB - 1; ++dd) xw[dd] = 0.0;
    // A long chain alternates its rows between two waves (bs_chain2: C5 back substitution 73 k -> 63 k
    // cycles); a short one stays on one wave (the hand-off costs more than it hides: C2 18.6 k -> 24.9 k).
    constexpr int kBs2Rows = 12;
    if (nd == 0) {
      if (NT >= kBs2Rows) {
        if (wave < 2) bs_chain2<false>(Wg, zp, xs, rdone, NT - 1, 0, xw, NT, wave, lane, li, lk, tmo);
      } else if (wave == 0) {
        bs_chain<false>(Wg, zp, xs, NT - 1, 0, xw, NT, lane, li, lk);
      }
    } else {
      // separator rows (one wave), then A (waves 0, 1) beside B (waves 2, 3, reversed)
      if (wave == 0) bs_chain<false>(Wg, zp, xs, m + 6, m, xw, NT, lane, li, lk);
      __syncthreads();
      if (wave < 2) {
#pragma unroll
        for (int dd = 1; dd < kTB; ++dd) xw[dd - 1] = xs[16 * (m - 1 + dd) + li];
        if (m >= kBs2Rows)
          bs_chain2<false>(Wg, zp, xs, rdone, m - 1, 0, xw, NT, wave, lane, li, lk, tmo);
        else if (wave == 0)
          bs_chain<false>(Wg, zp, xs, m - 1, 0, xw, NT, lane, li, lk);
      } else if (wave < 4) {
        // x of reversed rows nd .. nd+6 (the separator, S tile rows m+6 .. m)
#pragma unroll
        for (int dd = 1; dd < kTB; ++dd) xw[dd - 1] = xs[16 * (NT - nd - dd) + 15 - li];
        if (nd >= kBs2Rows)
          bs_chain2<true>(Wg + (size_t)NT * kTB * 256, zpg, xs, rdone_b, nd - 1, 0, xw, NT, wave - 2, lane, li,
                          lk, tmo);
        else if (wave == 2)
          bs_chain<true>(Wg + (size_t)NT * kTB * 256, zpg, xs, nd - 1, 0, xw, NT, lane, li, lk);
      }
    }
  }
  if (tid == 0 && nd > 0) tflag[1] = epoch + 1;
  if (bad && lane == 0) sh.fail = 1;
  if (tmo && lane == 0) sh.tmo = 1;   // a separator or back-substitution hand-off that timed out
  SG_TSTAMP(5)
  __syncthreads();
  double* y = d.work;
  for (int i = tid; i < n; i += kTileThreads) {
    d.xc[i] = xs[i];
    y[i] = xs[i];
  }
  if (border) {   // k_chol_border reads the factor's status and runs the candidate pass
    if (tid == 0) {
      d.xchg_chol[kCFail] = sh.fail ? 1.0 : 0.0;
      d.xchg_chol[kCTimeout] = sh.tmo ? 1.0 : 0.0;
    }
    return;
  }
  if (!cand_lds) __syncthreads();
  if (cand_lds)
    chol_candidates_lds<kTileThreads>(d, xs, sh.fail, cl, cur, sh.tmo);
  else
    chol_candidates<kTileThreads>(d, xs, sh.fail, sh.tmo);
  SG_TSTAMP(6)
  if (kStamp && lane == 0 && wave < 2)
    for (int s_ = 0; s_ < 16; ++s_) d.stamps[16 * wave + s_] += tacc[s_];
}
#undef SG_TSTAMP

// ------------------------------------------------------------------------------------------------
// Bordered band solve: SolveAllFrames(..., true) (slam.cpp:447-480), free intrinsics.  S is an arrowhead: the
// frame part S_ff (order nf = kc0) keeps its co-visibility band and only the nk <= 16 intrinsics columns S_fk
// are dense.  k_chol_tiles factors S_ff = U^T U on its band (flags bit 3) and leaves, per tile row K, Z_K =
// U_KK^-T (slot 0 of the W row), W_KJ = U_KK^-1 U_KJ and x_f0 = S_ff^-1 r_f in xc.  With U = Db (I + W) (Db the
// diagonal tiles), this workgroup finishes by block elimination of the border:
//   (1) forward chain over the tile rows (one wave, the intrinsics as one 16-wide tile column):
//         v_K = S_KB - sum_{d=1..7} W_{K-d,K}^T v_{K-d},   w_K = Z_K v_K   (w = U^-T S_fk),
//       C = S_kk - sum_K w_K^T w_K, and q_K = Z_K^T w_K kept for step (3); four MFMAs per tile product;
//   (2) beside it, the other waves form r_k - S_kf x_f0; then x_k = C^-1 (r_k - S_kf x_f0) (one wave, column
//       per lane);
//   (3) t = S_ff^-1 S_fk x_k = U^-1 (w x_k) by the band back substitution (bs_chain over the same W tiles with
//       z'_K = q_K x_k), and x_f = x_f0 - t;
//   (4) the candidate pass (chol_candidates) on x, as k_chol_tiles would have run it.
// The same elimination as k_cholesky_global's arrowhead factorisation, reordered: equal up to rounding.
constexpr int kBordThreads = 256;
// Dynamic LDS (doubles): x [16 NT], z' [16 NT], row flags [NT ints], then (flags bit 0) the q_K tiles [256 NT] and
// (bit 1) the candidate pass's operands (CandLds, staged by the waves that wait for the chain).
static inline size_t border_lds_doubles(int NT, int flags, int F, int D, int n) {
  size_t o = 32 * (size_t)NT + (NT + 1) / 2;
  if (flags & 1) o += 256 * (size_t)NT;
  if (flags & 2) o += (CandLds::bytes(F, D, n) + 7) / 8;
  return o;
}
template <bool kQlds>   // (flags bit 0 as a template parameter: a run-time choice of LDS or global compiles to flat accesses)
__global__ __launch_bounds__(kBordThreads) void k_chol_border(Dev d, double* __restrict__ Wg, int flags) {
  const LmState* st = d.st;
  if (st->done) return;
  extern __shared__ double bdyn[];
  const int n = d.n, nf = d.kc0, nk = n - nf, NT = (nf + 15) >> 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lk = lane >> 4;
  const bool cand_lds = (flags & 2) != 0;
  double* xs = bdyn;                                   // [16 NT] t, then x_f
  double* zq = bdyn + 16 * NT;                         // [16 NT] q_K x_k
  int* rdone = reinterpret_cast<int*>(bdyn + 32 * NT);   // [NT] bs_chain2 row flags
  size_t off = 32 * (size_t)NT + (NT + 1) / 2;
  // q_K tiles (acc layout): LDS, or the dissected bottom's W space.  Two pointers and a uniform branch at each
  // use, never one pointer that may be either (that compiles to flat accesses, which wait on both counters)
  constexpr bool qlds = kQlds;
  double* Ql = bdyn + off;
  double* Qg = Wg + (size_t)NT * kTB * 256;
  if (qlds) off += 256 * (size_t)NT;
  CandLds cl;
  cl.carve(bdyn + off, d.F, d.D, n);
  const double* S = d.S;
  const double* xc = d.xc;                             // x_f0 (frame rows), r_k (border rows)
  __shared__ double Cs[16][kTLd];
  __shared__ double rk[16], xk[16], rpart[kBordThreads / 64][16];
  __shared__ double Ids[16 * kTLd], prw[2 * kCholNb];   // tile_factor's identity tile and pivot-row scratch
  for (int i = tid; i < 16 * kTLd; i += kBordThreads) Ids[i] = (i / kTLd == i % kTLd) ? 1.0 : 0.0;
  __shared__ int bad_sh;
  // SG_STAMP=1: thread 0's s_memtime after each step, the deltas accumulated over launches in d.stamps[40 + k]
  // at the end (no global access between the stamps)
  unsigned long long tst[10];
  // (asm volatile with a memory clobber: the builtin may be scheduled across the code it should bracket)
  auto now_t = []() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
    return t;
  };
  tst[0] = now_t();
  auto bstamp = [&](int k) { tst[k + 1] = now_t(); };
  for (int k = 1; k < 10; ++k) tst[k] = tst[0];
  const int fail0 = d.xchg_chol[kCFail] != 0.0, tmo0 = d.xchg_chol[kCTimeout] != 0.0;
  for (int k = tid; k < NT; k += kBordThreads) rdone[k] = 0;
  if (tid == 0) bad_sh = fail0;
  // (1) the forward chain on four waves, handing tiles over through LDS rings behind monotonic flags:
  //   wave 0 (the chain): v_K = S_KB + F_K - W_{K-2,K}^T v_{K-2} - W_{K-1,K}^T v_{K-1}, w_K = Z_K v_K; posts
  //     v_K, w_K (vpost = K);
  //   waves 1, 2: the far terms F_K = -sum W_{K-d,K}^T v_{K-d}, d in {3, 4, 5} / {6, 7}, up to three rows ahead
  //     of the chain (they need v up to K-3), posted per row (fpost[h] = K);
  //   wave 3: C -= w_K^T w_K and q_K = Z_K^T w_K from the posted w_K (wdone = K).
  // So the chain's own matrix-core work per row is 12 MFMAs (was 40 on one SIMD).  Ring safety: v slot K & 7 is
  // rewritten at row K + 8 after F_{K+7} was consumed; F slot K & 3 at row K + 4 after the chain used F_K; w
  // slot K & 3 at row K + 4 after wave 3 took w_K.  Bounded waits (a time-out is reported as kCTimeout).
  __shared__ double vring[8][256], wring[4][256], fring[2][4][256];
  __shared__ int vpost, fpost[2], wdone;
  if (tid == 0) {
    vpost = -1;
    fpost[0] = fpost[1] = -1;
    wdone = -1;
  }
  __syncthreads();
  bool tmo_chain = false;
  // The rings and flags are LDS, whose accesses from one wave execute in order: data then flag on the writer,
  // flag then data on the reader need only compiler barriers — no fence, which would also wait for this wave's
  // outstanding global loads (the next row's prefetch) on every post.
  auto wait_ge = [&](int* flag, int v) {
    int spin = 0;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < v && ++spin < kLaSpinMax)
      __builtin_amdgcn_s_sleep(0);
    tmo_chain |= spin >= kLaSpinMax;
    asm volatile("" ::: "memory");
  };
  auto post = [&](int* flag, int v) {
    asm volatile("" ::: "memory");
    if (lane == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  const f64x4 zero = {0.0, 0.0, 0.0, 0.0};
  if (wave == 0) {
    // row K's operands (S_KB, W_{K-1,K}, Z_K) loaded one row ahead; unconditional loads (an index selected, not a
    // value: S's zero constant past the system; row -1's W tile multiplies the zero v_{-1})
    struct RowOps {
      double sb[4], w1[4], w2[4], za[4];
    };
    auto row_load = [&](RowOps& o, int K) {
      const int Kc = min(K, NT - 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * Kc + lk + 4 * q;
        o.sb[q] = S[(r < nf && li < nk) ? (size_t)r * n + nf + li : (size_t)n * n + n];
      }
      const double* wt = Wg + ((size_t)max(Kc - 1, 0) * kTB + 1) * 256 + lane;
      const double* wt2 = Wg + ((size_t)max(Kc - 2, 0) * kTB + 2) * 256 + lane;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        o.w1[s4] = -wt[s4 * 64];
        o.w2[s4] = -wt2[s4 * 64];
      }
      const double* Z = Wg + (size_t)Kc * kTB * 256;   // row-major Z_K
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) o.za[s4] = Z[li * 16 + 4 * s4 + lk];   // Z^T in acc layout: Z v
    };
    f64x4 vprev = zero, vprev2 = zero;
    RowOps ops[2];
    row_load(ops[0], 0);
    auto row = [&](RowOps& o, int K) {
      f64x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = o.sb[q];
      v = mfma_f64_k16(o.w2, vprev2, v);   // d = 2, then d = 1 (the helpers hold d >= 3: three rows of slack)
      v = mfma_f64_k16(o.w1, vprev, v);
      wait_ge(&fpost[0], K);
      wait_ge(&fpost[1], K);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += fring[0][K & 3][q * 64 + lane] + fring[1][K & 3][q * 64 + lane];
      const f64x4 w = mfma_f64_k16(o.za, v, zero);
      if (K >= 4) wait_ge(&wdone, K - 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        vring[K & 7][q * 64 + lane] = v[q];
        wring[K & 3][q * 64 + lane] = w[q];
      }
      post(&vpost, K);
      vprev2 = vprev;
      vprev = v;
    };
#pragma nounroll
    for (int K = 0; K < NT; K += 2) {
      row_load(ops[1], K + 1);
      row(ops[0], K);
      if (K + 1 < NT) {
        row_load(ops[0], K + 2);
        row(ops[1], K + 1);
      }
    }
  } else if (wave <= 2) {
    // far terms, d in {3, 4, 5} (wave 1) or {6, 7} (wave 2); W tiles one row ahead
    const int h = wave - 1, d0 = 3 + 3 * h;
    double wn[2][3][4];
    auto wload = [&](double (&o)[3][4], int K) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int dj = min(d0 + j, kTB - 1);   // (wave 2's third slot is past the band: loaded, never used)
        const double* wt = Wg + ((size_t)max(K - dj, 0) * kTB + dj) * 256 + lane;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) o[j][s4] = -wt[s4 * 64];
      }
    };
    // (buffers by compile-time index: the loop is unrolled by two, a run-time index would put them in scratch)
    auto hrow = [&](double (&wc)[3][4], double (&wnx)[3][4], int K) {
      if (K + 1 < NT) wload(wnx, K + 1);
      // v up to K - d0 posted, and F slot K & 3 free (the chain has used F_{K-4})
      wait_ge(&vpost, max(K - d0, K - 4));
      f64x4 f = zero;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int Kv = K - (d0 + j);
        if (Kv >= 0 && d0 + j < kTB) {
          f64x4 vt;
#pragma unroll
          for (int q = 0; q < 4; ++q) vt[q] = vring[Kv & 7][q * 64 + lane];
          f = mfma_f64_k16(wc[j], vt, f);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) fring[h][K & 3][q * 64 + lane] = f[q];
      post(&fpost[h], K);
    };
    wload(wn[0], 0);
#pragma nounroll
    for (int K = 0; K < NT; K += 2) {
      hrow(wn[0], wn[1], K);
      if (K + 1 < NT) hrow(wn[1], wn[0], K + 1);
    }
  } else {
    // C and the q_K tiles from the posted w_K
    f64x4 C;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = lk + 4 * q, c = li;
      const int a = min(r, c), b = max(r, c);   // S_kk upper triangle
      C[q] = (r < nk && c < nk) ? S[(size_t)(nf + a) * n + nf + b] : (r == c ? 1.0 : 0.0);
    }
    double zb[2][4];
    auto zload = [&](double (&o)[4], int K) {
      const double* Z = Wg + (size_t)min(K, NT - 1) * kTB * 256;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) o[s4] = Z[(4 * s4 + lk) * 16 + li];   // Z in acc layout: Z^T w
    };
    auto crow = [&](double (&zc)[4], double (&znx)[4], int K) {
      zload(znx, K + 1);
      wait_ge(&vpost, K);
      f64x4 w;
      double wn4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w[q] = wring[K & 3][q * 64 + lane];
        wn4[q] = -w[q];
      }
      post(&wdone, K);
      C = mfma_f64_k16(wn4, w, C);
      const f64x4 qv = mfma_f64_k16(zc, w, zero);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr (qlds) Ql[(size_t)K * 256 + q * 64 + lane] = qv[q];
        else Qg[(size_t)K * 256 + q * 64 + lane] = qv[q];
      }
    };
    zload(zb[0], 0);
#pragma nounroll
    for (int K = 0; K < NT; K += 2) {
      crow(zb[0], zb[1], K);
      if (K + 1 < NT) crow(zb[1], zb[0], K + 1);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) Cs[lk + 4 * q][li] = (lk + 4 * q <= li) ? C[q] : 0.0;   // upper (tile_factor)
  }
  __syncthreads();
  // (2) S_kf x_f0 on every wave: a thread per frame row (a row's 14 border entries are contiguous), per-wave sums
  // per intrinsic, combined in wave order below
  {
    double part[kCholNb];
#pragma unroll
    for (int c = 0; c < kCholNb; ++c) part[c] = 0.0;
    for (int i = tid; i < nf; i += kBordThreads) {
      const double xi = xc[i];
      const double* row = S + (size_t)i * n + nf;
#pragma unroll
      for (int c = 0; c < kCholNb; ++c) part[c] = fma(row[c], xi, part[c]);   // (c >= nk: unused, inside S)
    }
#pragma unroll
    for (int c = 0; c < kCholNb; ++c) {
      const double v = wave_sum_full(part[c]);
      if (lane == 0) rpart[wave][c] = v;
    }
  }
  if (d.stamps && tid == 0) bstamp(0);
  __syncthreads();
  if (d.stamps && tid == 0) bstamp(5);
  if (tid < kCholNb)
    rk[tid] = tid < nk ? xc[nf + tid] - (((rpart[0][tid] + rpart[1][tid]) + rpart[2][tid]) + rpart[3][tid]) : 0.0;
  __syncthreads();
  if (d.stamps && tid == 0) bstamp(6);
  if (wave == 0) {
    // x_k = C^-1 rk by the tiled Cholesky's 16x16 factorisation (tile_factor: the identity and rk as augmented
    // columns give Z = U_c^-T and z = Z rk), then x_k = Z^T z (lanes 16..31 hold Z's columns)
    double ca[kCholNb];
    const bool bad = tile_factor(&Cs[0][0], rk, Ids, prw, ca);
    double zr[kCholNb];
#pragma unroll
    for (int r = 0; r < kCholNb; ++r) zr[r] = readlane_d(ca[r], 32);
    if (lane >= 16 && lane < 32) {
      double x = 0.0;
#pragma unroll
      for (int r = 0; r < kCholNb; ++r) x = fma(ca[r], zr[r], x);
      xk[lane - 16] = lane - 16 < nk ? x : 0.0;
    }
    if (lane == 0 && bad) bad_sh = 1;
  }
  if (d.stamps && tid == 0) bstamp(1);
  __syncthreads();
  if (d.stamps && tid == 0) bstamp(7);
  // (3) z'_K = q_K x_k, then t = U^-1 (w x_k)
  for (int i = tid; i < 16 * NT; i += kBordThreads) {
    const int K = i >> 4, r = i & 15;
    const size_t qo = (size_t)K * 256 + (r >> 2) * 64 + (r & 3) * 16;
    double acc = 0.0;
    if constexpr (qlds) {
#pragma unroll
      for (int c = 0; c < kCholNb; ++c) acc = fma(Ql[qo + c], xk[c], acc);   // (columns >= nk: zero in q and x_k)
    } else {
#pragma unroll
      for (int c = 0; c < kCholNb; ++c) acc = fma(Qg[qo + c], xk[c], acc);
    }
    zq[i] = acc;
  }
  if (d.stamps && tid == 0) bstamp(2);
  __syncthreads();
  if (d.stamps && tid == 0) bstamp(8);
  bool tmo = tmo0 || tmo_chain;
  {
    double xw[kTB - 1];
#pragma unroll
    for (int dd = 0; dd < kTB - 1; ++dd) xw[dd] = 0.0;
    constexpr int kBs2Rows = 12;
    const int nbs = NT >= kBs2Rows ? 2 : 1;   // waves on the back substitution; the others stage the candidates
    if (NT >= kBs2Rows) {
      if (wave < 2) bs_chain2<false>(Wg, zq, xs, rdone, NT - 1, 0, xw, NT, wave, lane, li, lk, tmo);
    } else if (wave == 0) {
      bs_chain<false>(Wg, zq, xs, NT - 1, 0, xw, NT, lane, li, lk);
    }
    if (wave >= nbs && cand_lds) cand_prefetch(d, cl, st->cur, tid - 64 * nbs, kBordThreads - 64 * nbs);
  }
  __shared__ int tmo_sh;
  if (tid == 0) tmo_sh = 0;
  if (d.stamps && tid == 0) bstamp(3);
  __syncthreads();
  if (tmo && lane == 0) tmo_sh = 1;
  // (4) x = (x_f0 - t, x_k): xc, the solution copy in work, and the candidate pass
  double* y = d.work;
  for (int i = tid; i < n; i += kBordThreads) {
    const double x = i < nf ? xc[i] - xs[i] : xk[i - nf];
    if (i < nf) xs[i] = x;
    d.xc[i] = x;
    y[i] = x;
  }
  __syncthreads();
  if (cand_lds)
    chol_candidates_lds<kBordThreads>(d, xs, bad_sh, cl, st->cur, tmo_sh);
  else
    chol_candidates<kBordThreads>(d, xs, bad_sh, tmo_sh);
  if (d.stamps && tid == 0) {
    bstamp(4);
    // stamps[48 + k]: time from the start to stamp k (0 chain, 5 after B1, 6 after B2, 1 C solve, 7 after B3,
    // 2 z', 8 after B4, 3 back substitution, 4 end), accumulated over launches
#pragma unroll
    for (int k = 1; k < 10; ++k) d.stamps[48 + k - 1] += tst[k] - tst[0];   // (slots 32-45: k_schur's)
  }
}

// ------------------------------------------------------------------------------------------------
// k_point_update: back-substitution x_p = V~^-1 (g~_p - A_p^T A_c x_c), model cost change
// -(A s).(r + A s / 2), candidate point X+ = X - S_p x_p and the candidate reprojection cost.
// Same work decomposition as k_linearize (one wave per LinChunk, one observation per lane, rounds of
// whole points): each observation's record is read once; per round
//   1. lane per observation: u = A_c x_c, and A_p^T u into the LDS accumulator of its point;
//   2. lane per point: x_p, X+, |step|^2, |X+|^2;
//   3. lane per observation: the model term and the candidate projection at X+ (project.h).
// A wide chunk (one point over several rounds) runs pass 1 over all its pieces, then 2, then 3.
struct PuObs {
  double r[2], Jp[8], u[2];
  int f, b, cam;
  bool on;   // a non-fixed observation of this round
};

// pacc == nullptr: the records only (a wide chunk's second walk).
__device__ __forceinline__ void pu_pass1(const Dev& d, int cur, const LinRound& R, int lane, double* pacc, PuObs& ob) {
  ob.on = false;
  const int nc = R.o1 - R.o0;
  if (lane >= nc) return;
  const int o = R.o0 + lane;
  const int m = d.obs_meta[o];
  const int p = d.obs_pnt[o];
  ob.f = d.obs_frame[o];
  if (m & kMetaFixed) return;
  ob.on = true;
  ob.b = meta_block(m);
  ob.cam = meta_cam(m);
  const double4 s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
  const double sp[4] = {s4.x, s4.y, s4.z, s4.w};
  double Jc[12];
  load_scaled_J(d, d.J[cur], o, ob.b, sp, ob.r, Jc, ob.Jp);
  ob.u[0] = ob.u[1] = 0.0;
  if (ob.b >= 0) {
    const double* xc = d.xc + 6 * ob.b;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      ob.u[0] += Jc[c] * xc[c];
      ob.u[1] += Jc[6 + c] * xc[c];
    }
  }
  if (d.nk) {   // free intrinsics: u += A_k x_k
    const double* Jk = d.Jk + 14 * (size_t)o;
    const int kc = d.kc0 + 7 * ob.cam;
    for (int c = 0; c < 7; ++c) {
      const double xs = d.xc[kc + c] * d.scale_c[kc + c];
      ob.u[0] += Jk[c] * xs;
      ob.u[1] += Jk[7 + c] * xs;
    }
  }
  if (ob.b >= 0 || d.nk) {
    if (pacc && (m & kMetaPfree)) {
      double* pa = pacc + (p - R.p0) * 4;
#pragma unroll
      for (int a = 0; a < 4; ++a) atomicAdd(pa + a, ob.Jp[a] * ob.u[0] + ob.Jp[4 + a] * ob.u[1]);
    }
  }
}

__device__ __forceinline__ void pu_pass3(const Dev& d, const LinRound& R, int lane, int nxt, const double* xps,
                                         const double* Xns, const PuObs& ob, double& model, double& candcost,
                                         double& candfail) {
  if (!ob.on) return;
  const int o = R.o0 + lane;
  const int lp = d.obs_pnt[o] - R.p0;
  const double* xp = xps + 4 * lp;
  double m0 = -ob.u[0], m1 = -ob.u[1];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    m0 -= ob.Jp[c] * xp[c];
    m1 -= ob.Jp[4 + c] * xp[c];
  }
  model -= m0 * (ob.r[0] + 0.5 * m0) + m1 * (ob.r[1] + 0.5 * m1);
  const double Xn[4] = {Xns[4 * lp], Xns[4 * lp + 1], Xns[4 * lp + 2], Xns[4 * lp + 3]};
  double uv[2] = {0.0, 0.0};
  const bool okp = Project(d.q[nxt] + 4 * ob.f, d.t[nxt] + 3 * ob.f, d.k[nxt] + 7 * ob.cam, Xn, uv);
  const double2 pt = reinterpret_cast<const double2*>(d.obs_pt)[o];
  const double e0 = uv[0] - pt.x, e1 = uv[1] - pt.y;
  double rho0, rho1;
  Cauchy(e0 * e0 + e1 * e1, d.b, d.inv_b, &rho0, &rho1);
  // both accumulators updated unconditionally (selects, no early return): a conditional update of one of
  // two references made the compiler keep them in an indexed stack slot (scratch traffic on every lane)
  candfail += okp ? 0.0 : 1.0;
  candcost += okp ? 0.5 * rho0 : 0.0;
}

// pass 2 for the points [p0, p1) of a round (lane per point): x_p, X+ into LDS and HBM.
__device__ __forceinline__ void pu_pass2(const Dev& d, int p0, int p1, int lane, int cur, int nxt, double* pacc,
                                         double* xps, double* Xns, double& step2, double& candx2) {
  if (lane >= p1 - p0) return;
  const int p = p0 + lane;
  const bool pf = d.pfree[p] != 0;
  const double4 Xv = reinterpret_cast<const double4*>(d.X[cur])[p];
  const double X[4] = {Xv.x, Xv.y, Xv.z, Xv.w};
  double* pa = pacc + 4 * lane;
  double xp[4] = {0.0, 0.0, 0.0, 0.0}, Xn[4] = {X[0], X[1], X[2], X[3]};
  if (pf) {
    const double4 s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
    const double sp[4] = {s4.x, s4.y, s4.z, s4.w};
    const double4 g4 = reinterpret_cast<const double4*>(d.g[cur])[p];
    const double rhs[4] = {g4.x * sp[0] - pa[0], g4.y * sp[1] - pa[1], g4.z * sp[2] - pa[2], g4.w * sp[3] - pa[3]};
    const double* Vi = d.Vinv + 10 * (size_t)p;
    double Vl[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) Vl[i] = Vi[i];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) s += sym4(Vl, a, c) * rhs[c];
      xp[a] = s;
    }
    // step s_p = -x_p (scaled); candidate X+ = X + S_p s_p
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      Xn[a] = X[a] + (-xp[a] * sp[a]);
      step2 += (Xn[a] - X[a]) * (Xn[a] - X[a]);
      candx2 += Xn[a] * Xn[a];
    }
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    pa[a] = 0.0;
    xps[4 * lane + a] = xp[a];
    Xns[4 * lane + a] = Xn[a];
  }
  reinterpret_cast<double4*>(d.X[nxt])[p] = make_double4(Xn[0], Xn[1], Xn[2], Xn[3]);
}

__global__ __launch_bounds__(kLinThreads) void k_point_update(Dev d) {
  const LmState* st = d.st;
  if (st->done) return;
  const int cur = st->cur, nxt = cur ^ 1;
  // work unit: one round of a regular chunk (rounds are independent here: the camera step is known), or a
  // whole wide chunk (one point split over rounds)
  const int unit = d.pu_units[blockIdx.x];
  LinChunk ch;
  if (unit >= 0) {
    ch.r0 = unit;
    ch.r1 = unit + 1;
    ch.wide = 0;
  } else {
    ch = d.lchunks[-unit - 1];
  }
  __shared__ double pacc[kLinPts * 4], xps[kLinPts * 4], Xns[kLinPts * 4];
  const int lane = threadIdx.x;
  for (int i = lane; i < kLinPts * 4; i += kLinThreads) pacc[i] = 0.0;
  lds_fence_wave();
  double model = 0.0, candcost = 0.0, candfail = 0.0, step2 = 0.0, candx2 = 0.0;
  if (!ch.wide) {
    for (int r = ch.r0; r < ch.r1; ++r) {
      const LinRound R = d.lrounds[r];
      PuObs ob;
      pu_pass1(d, cur, R, lane, pacc, ob);
      lds_fence_wave();
      pu_pass2(d, R.p0, R.p1, lane, cur, nxt, pacc, xps, Xns, step2, candx2);
      lds_fence_wave();
      pu_pass3(d, R, lane, nxt, xps, Xns, ob, model, candcost, candfail);
      lds_fence_wave();
    }
  } else {
    for (int r = ch.r0; r < ch.r1; ++r) {
      PuObs ob;
      pu_pass1(d, cur, d.lrounds[r], lane, pacc, ob);
    }
    lds_fence_wave();
    pu_pass2(d, ch.p0, ch.p1, lane, cur, nxt, pacc, xps, Xns, step2, candx2);
    lds_fence_wave();
    for (int r = ch.r0; r < ch.r1; ++r) {
      const LinRound R = d.lrounds[r];
      PuObs ob;
      pu_pass1(d, cur, R, lane, nullptr, ob);
      pu_pass3(d, R, lane, nxt, xps, Xns, ob, model, candcost, candfail);
    }
  }
  model = wave_sum_full(model);
  candcost = wave_sum_full(candcost);
  candfail = wave_sum_full(candfail);
  step2 = wave_sum_full(step2);
  candx2 = wave_sum_full(candx2);
  if (lane == 0) {
    double* sc = d.chunk_scal + blockIdx.x;   // structure of arrays: slot j at [j * npu + unit]
    const size_t ns = d.npu;
    sc[kModel * ns] = model;
    sc[kCandCost * ns] = candcost;
    sc[kCandFail * ns] = candfail;
    sc[kStep2 * ns] = step2;
    sc[kCandX2 * ns] = candx2;
  }
}

// ------------------------------------------------------------------------------------------------
// k_update_lin: k_point_update fused with the next linearization (speculative linearization).  The candidate
// pass projects every observation at x+ = x[cur ^ 1] anyway; here it evaluates the analytic Jacobian there too
// and writes the candidate's J records, point blocks V / g and camera partials into the other slot (J, V, g,
// cam_slab, cam_wide, lin_scal [cur ^ 1]).  When the decision accepts the step, cur flips and that slot is the
// current linearization — Ceres evaluates the Jacobian at the accepted x (slam.cpp:482-521), the same arithmetic
// at the same point — so no k_linearize launch and no second sweep over the observations follow; a rejected
// step leaves slot cur as it was (the next iteration re-reduces it when it must re-linearize).
// Work decomposition: k_linearize's chunks (the candidate camera partials in k_linearize's order), and the
// update scalars per round (k_point_update's units, in its lane order), so the solve is bitwise the one of
// k_point_update + k_linearize (test_ba_gpu.py::test_speculative_linearization_is_bitwise_identical).

// One lane's observation of round R: the model term of the current linearization (ob, from pass 1), then
// project.h + analytic Jacobian + Cauchy corrector at the candidate (k_linearize's body at x[nxt]): the J
// record into slot nxt, the candidate's point and camera terms into LDS, its cost.
__device__ __forceinline__ void ul_obs(const Dev& d, const LinRound& R, const LinChunk& ch, int lane, int nxt,
                                       const PuObs& ob, const double* xps, const double* Xns, double* pacc,
                                       double* camacc, double (*lsum)[kLinThreads], double& model, double& cost,
                                       double& candcost, double& candfail) {
  if (lane >= R.o1 - R.o0) return;
  const int o = R.o0 + lane;
  const int m = d.obs_meta[o];
  const int lp = d.obs_pnt[o] - R.p0;
  const int f = d.obs_frame[o];
  const bool fx = (m & kMetaFixed) != 0;
  if (ob.on) {   // k_point_update pass 3: -(A s).(r + A s / 2)
    const double* xp = xps + 4 * lp;
    double m0 = -ob.u[0], m1 = -ob.u[1];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      m0 -= ob.Jp[c] * xp[c];
      m1 -= ob.Jp[4 + c] * xp[c];
    }
    model -= m0 * (ob.r[0] + 0.5 * m0) + m1 * (ob.r[1] + 0.5 * m1);
  }
  const double X[4] = {Xns[4 * lp], Xns[4 * lp + 1], Xns[4 * lp + 2], Xns[4 * lp + 3]};
  const double2 uv = reinterpret_cast<const double2*>(d.obs_pt)[o];
  const double pt[2] = {uv.x, uv.y};
  double rr[2], Jc[12], Jp[8], c;
  const bool ok = LinearizeObservation(d.q[nxt] + 4 * f, d.t[nxt] + 3 * f, d.k[nxt] + 7 * meta_cam(m), X, pt, d.b,
                                       d.inv_b, rr, Jc, Jp, &c);
  // the candidate cost as k_point_update sums it (c is project.h's forward value: the same bits as Project)
  if (!fx) {
    candfail += ok ? 0.0 : 1.0;
    candcost += ok ? c : 0.0;
  }
  double2* Jo = reinterpret_cast<double2*>(d.J[nxt]) + jidx2(o, 0);   // pair e2 at Jo[64 e2]
  if (!ok || fx) {
    if (!ok) lsum[fx ? 1 : 0][lane] += 1.0;   // (a fixed observation's cost counts at iteration 0 only)
#pragma unroll
    for (int i = 0; i < kJStride / 2; ++i) Jo[64 * i] = make_double2(0.0, 0.0);
    return;
  }
  cost += c;
  const bool pf = (m & kMetaPfree) != 0;
  const int b = meta_block(m);
  if (b < 0) {
#pragma unroll
    for (int i = 0; i < 12; ++i) Jc[i] = 0.0;
  } else {
    if (!(m & kMetaRot)) { Jc[0] = Jc[1] = Jc[2] = Jc[6] = Jc[7] = Jc[8] = 0.0; }
    if (!(m & kMetaTrans)) { Jc[3] = Jc[4] = Jc[5] = Jc[9] = Jc[10] = Jc[11] = 0.0; }
  }
  if (!pf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) Jp[i] = 0.0;
  }
  Jo[0] = make_double2(rr[0], rr[1]);
#pragma unroll
  for (int i = 0; i < 6; ++i) Jo[64 * (1 + i)] = make_double2(Jc[2 * i], Jc[2 * i + 1]);
#pragma unroll
  for (int i = 0; i < 4; ++i) Jo[64 * (7 + i)] = make_double2(Jp[2 * i], Jp[2 * i + 1]);
  Jo[64 * 11] = make_double2(c, 0.0);
  if (pf) {
    double* pa = pacc + lp * 14;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
#pragma unroll
      for (int cc = 0; cc < 4; ++cc)
        if (cc >= a) atomicAdd(pa + u4(a, cc), Jp[a] * Jp[cc] + Jp[4 + a] * Jp[4 + cc]);
      atomicAdd(pa + 10 + a, Jp[a] * rr[0] + Jp[4 + a] * rr[1]);
    }
  }
  if (b >= 0) {
    auto add_cam = [&](double* dst) {
#pragma unroll
      for (int a = 0; a < 6; ++a) {
#pragma unroll
        for (int cc = 0; cc < 6; ++cc)
          if (cc >= a) atomicAdd(dst + u6(a, cc), Jc[a] * Jc[cc] + Jc[6 + a] * Jc[6 + cc]);
        atomicAdd(dst + 21 + a, Jc[a] * rr[0] + Jc[6 + a] * rr[1]);
      }
    };
    if (ch.wide) add_cam(d.cam_wide[nxt] + (size_t)b * kCamV);
    else add_cam(camacc + (b - ch.b_lo) * kCamV);
  }
}

// The candidate point blocks of the points [p0, p1) (lane per point) into slot nxt (k_linearize's point pass).
__device__ __forceinline__ void ul_points(const Dev& d, int p0, int p1, int lane, int nxt, double* pacc,
                                          double& gmax) {
  if (lane >= p1 - p0) return;
  const int pp = p0 + lane;
  double* pa = pacc + lane * 14;
  double V[10], g[4];
#pragma unroll
  for (int i = 0; i < 10; ++i) V[i] = pa[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = pa[10 + i];
#pragma unroll
  for (int i = 0; i < 14; ++i) pa[i] = 0.0;
  double2* Vd = reinterpret_cast<double2*>(d.V[nxt] + 10 * (size_t)pp);
#pragma unroll
  for (int k = 0; k < 5; ++k) Vd[k] = make_double2(V[2 * k], V[2 * k + 1]);
  reinterpret_cast<double4*>(d.g[nxt])[pp] = make_double4(g[0], g[1], g[2], g[3]);
  if (d.pfree[pp]) gmax = fmax(gmax, fmax(fmax(fabs(g[0]), fabs(g[1])), fmax(fabs(g[2]), fabs(g[3]))));
}

// k_point_update's per-unit scalars (its wave sums, in its order), then reset for the next unit.
__device__ __forceinline__ void ul_unit_scalars(const Dev& d, int unit, int lane, double& model, double& candcost,
                                                double& candfail, double& step2, double& candx2) {
  const double m = wave_sum_full(model), cc = wave_sum_full(candcost), cf = wave_sum_full(candfail);
  const double s2 = wave_sum_full(step2), x2 = wave_sum_full(candx2);
  if (lane == 0) {
    double* sc = d.chunk_scal + unit;   // structure of arrays: slot j at [j * npu + unit]
    const size_t ns = d.npu;
    sc[kModel * ns] = m;
    sc[kCandCost * ns] = cc;
    sc[kCandFail * ns] = cf;
    sc[kStep2 * ns] = s2;
    sc[kCandX2 * ns] = x2;
  }
  model = candcost = candfail = step2 = candx2 = 0.0;
}

template <bool kStamp, int kW>
__global__ __launch_bounds__(kLinThreads * kW) SG_LIN_ATTR void k_update_lin(Dev d) {
  const LmState* st = d.st;
  if (st->done) return;
  const int cur = st->cur, nxt = cur ^ 1;
  const LinChunk ch = d.lchunks[blockIdx.x];
  if (blockIdx.x == 0 && threadIdx.x == 0) d.st->spec_slot = nxt;   // (k_cam_reduce mode 1 reads it)
  // per wave (k_linearize's split of the chunk's rounds over its waves):
  __shared__ double pacc_w[kW][kLinPts * 14];         // candidate point blocks of the round: V (10) | g (4)
  __shared__ double camacc_w[kW][kLinNbMax * kCamV];  // candidate camera blocks of the window
  __shared__ double lsum_w[kW][2][kLinThreads];       // candidate failures: free, fixed observations
  __shared__ double ua_w[kW][kLinPts * 4], xps_w[kW][kLinPts * 4], Xns_w[kW][kLinPts * 4];
  __shared__ double wscal[8];                         // wave 1's chunk scalars
  const int lane = threadIdx.x & (kLinThreads - 1), wv = threadIdx.x / kLinThreads;
  double* pacc = pacc_w[wv];
  double* camacc = camacc_w[wv];
  double(*lsum)[kLinThreads] = lsum_w[wv];
  double* ua = ua_w[wv];     // A_p^T A_c x_c per point
  double* xps = xps_w[wv];   // x_p
  double* Xns = Xns_w[wv];   // X+
  const int ncv = ch.nb * kCamV;
  for (int i = lane; i < ncv; i += kLinThreads) camacc[i] = 0.0;
  for (int i = lane; i < kLinPts * 14; i += kLinThreads) pacc[i] = 0.0;
  for (int i = lane; i < kLinPts * 4; i += kLinThreads) ua[i] = 0.0;
  lsum[0][lane] = 0.0;
  lsum[1][lane] = 0.0;
  lds_fence_wave();
  double cost = 0.0, gmax = 0.0;
  double model = 0.0, candcost = 0.0, candfail = 0.0, step2 = 0.0, candx2 = 0.0;
  // SG_STAMP=1 (the kStamp build): lane 0 of the mid-grid and the last workgroup time their steps
  // (d.stamps[kUlStamp + 8 w + k])
  const int stw = !kStamp || !d.stamps || threadIdx.x != 0 ? -1
                  : blockIdx.x == gridDim.x / 2 ? 0 : blockIdx.x == gridDim.x - 1 ? 1 : -1;
  unsigned long long tl = 0;
  auto ul_stamp = [&](int k) {
    if (stw < 0) return;
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
    if (k >= 0) d.stamps[kUlStamp + 8 * stw + k] += t - tl;
    tl = t;
  };
  ul_stamp(-1);
  if (!ch.wide) {
    for (int r = ch.r0 + wv; r < ch.r1; r += kW) {
      const LinRound R = d.lrounds[r];
      PuObs ob;
      pu_pass1(d, cur, R, lane, ua, ob);
      lds_fence_wave();
      ul_stamp(0);
      pu_pass2(d, R.p0, R.p1, lane, cur, nxt, ua, xps, Xns, step2, candx2);
      lds_fence_wave();
      ul_stamp(1);
      ul_obs(d, R, ch, lane, nxt, ob, xps, Xns, pacc, camacc, lsum, model, cost, candcost, candfail);
      lds_fence_wave();
      ul_stamp(2);
      ul_points(d, R.p0, R.p1, lane, nxt, pacc, gmax);
      lds_fence_wave();
      ul_stamp(3);
      ul_unit_scalars(d, ch.u0 + (r - ch.r0), lane, model, candcost, candfail, step2, candx2);
      ul_stamp(4);
    }
  } else if (wv == 0) {
    // one point over several rounds: its back substitution needs every piece's A_p^T u first
    for (int r = ch.r0; r < ch.r1; ++r) {
      PuObs ob;
      pu_pass1(d, cur, d.lrounds[r], lane, ua, ob);
    }
    lds_fence_wave();
    pu_pass2(d, ch.p0, ch.p1, lane, cur, nxt, ua, xps, Xns, step2, candx2);
    lds_fence_wave();
    for (int r = ch.r0; r < ch.r1; ++r) {
      const LinRound R = d.lrounds[r];
      PuObs ob;
      pu_pass1(d, cur, R, lane, nullptr, ob);
      ul_obs(d, R, ch, lane, nxt, ob, xps, Xns, pacc, camacc, lsum, model, cost, candcost, candfail);
    }
    lds_fence_wave();
    ul_points(d, ch.p0, ch.p1, lane, nxt, pacc, gmax);
    lds_fence_wave();
    ul_unit_scalars(d, ch.u0, lane, model, candcost, candfail, step2, candx2);
  }
  lds_fence_wave();
  cost = wave_sum_full(cost);
  double fail = wave_sum_full(lsum[0][lane]);
  double ffail = wave_sum_full(lsum[1][lane]);
  gmax = wave_max_full(gmax);
  // the same combine as k_linearize's (its fixed and |X|^2 sums are zero here)
  double fixed = 0.0, xn2 = 0.0;
  lin_combine_waves<kW>(d.cam_slab[nxt] + ch.cam_off, camacc_w, ncv, wscal, wv, lane, cost, fail, fixed, ffail,
                        xn2, gmax);
  if (wv == 0 && lane == 0) {
    double* sc = d.lin_scal[nxt] + blockIdx.x;   // k_linearize's scalars of the candidate (never iteration 0)
    const size_t ns = d.nlin;
    sc[kCost * ns] = cost;
    sc[kFail * ns] = fail;
    sc[kFixed * ns] = 0.0;
    sc[kFixedFail * ns] = ffail;
    sc[kXnorm2 * ns] = 0.0;
    sc[kGmax * ns] = gmax;
  }
  ul_stamp(5);
  if (stw >= 0) d.stamps[kUlStamp + 8 * stw + 6] += 1;   // launches stamped
}

__device__ void decide_step(LmState& s, const double* u, const double* c);

// fuse: single rank, no all-reduce in between: thread 0 also runs k_decide's step (one launch less).
__global__ __launch_bounds__(kRedThreads) void k_upd_reduce(Dev d, int fuse) { upd_reduce_body(d, fuse); }

__device__ void upd_reduce_body(const Dev& d, int fuse) {
  const LmState* st = d.st;
  const int done = st->done;   // tested after the scalar loads are out (see k_S_reduce)
  __shared__ double red[kRedThreads / 64 * kUNum];
  const int tid = threadIdx.x;
  // the decision's inputs are loaded up front (one round trip overlapping the reduction, not a chain of
  // dependent ones after it), into LDS: thread 0's register copy of LmState beside the reduction's loads in
  // flight spilled (this body shares k_cam_reduce's 1024-thread, 128-VGPR budget)
  __shared__ LmState s;
  __shared__ double cc[kCNum];
  if (fuse && tid == 0) {
    s = *st;
    for (int j = 0; j < kCNum; ++j) cc[j] = d.xchg_chol[j];
  }
  double v[kUNum] = {};
  // the Cholesky's hand-off time-outs ride in the scalar exchange, so every shard ends the solve together
  if (tid == 0) v[kUTimeout] = d.xchg_chol[kCTimeout];
  constexpr int kUpdU = 4;   // work units' loads in flight per thread (8 measured slower)
  for (int c0 = tid; c0 < d.npu; c0 += kUpdU * kRedThreads) {
    double t[kUpdU][5];
#pragma unroll
    for (int u = 0; u < kUpdU; ++u) {
      const int c = c0 + u * kRedThreads;
      const double* sc = d.chunk_scal + (c < d.npu ? c : 0);   // coalesced: slot j at [j * npu + unit]
      const size_t ns = d.npu;
      t[u][0] = sc[kModel * ns];
      t[u][1] = sc[kCandCost * ns];
      t[u][2] = sc[kCandFail * ns];
      t[u][3] = sc[kStep2 * ns];
      t[u][4] = sc[kCandX2 * ns];
    }
#pragma unroll
    for (int u = 0; u < kUpdU; ++u)
      if (c0 + u * kRedThreads < d.npu) {
        v[kUModel] += t[u][0];
        v[kUCandCost] += t[u][1];
        v[kUCandFail] += t[u][2];
        v[kUStep2] += t[u][3];
        v[kUCandX2] += t[u][4];
      }
  }
  for (int g = tid; g < d.nseg + d.nwide; g += kRedThreads) v[kULinFail] += d.seg_fail[g];
  if (done) return;
  block_sum_multi_t0<kRedThreads, kUNum>(v, red);
  if (tid == 0) {
#pragma unroll
    for (int j = 0; j < kUNum; ++j) d.xchg_upd[j] = v[j];
    if (fuse) {
      decide_step(s, v, cc);
      *d.st = s;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// k_decide: TrustRegionMinimizer + LevenbergMarquardtStrategy step bookkeeping (Ceres 1.8 semantics).
// take (speculative chain): the accepted candidate's camera blocks and scalars (k_cam_reduce mode 1) become this
// rank's current ones, and the all-reduce buffer holds this rank's current blocks again (the camera-block
// all-reduce of landmark shards sums it in place).  256 threads.
__global__ void k_decide(Dev d, int take) {
  __shared__ int acc_sh;
  if (threadIdx.x == 0) {
    LmState s = *d.st;
    double u[kUNum], c[kCNum];
    for (int j = 0; j < kUNum; ++j) u[j] = d.xchg_upd[j];
    for (int j = 0; j < kCNum; ++j) c[j] = d.xchg_chol[j];
    const int c0 = s.cur;
    decide_step(s, u, c);
    acc_sh = s.cur != c0;
    if (take) s.accepted = 0;
    *d.st = s;
  }
  if (!take) return;
  __syncthreads();
  const int nx = d.NB * kCamV + kXNum + d.nranks;
  const bool acc = acc_sh != 0;
  for (int i = threadIdx.x; i < nx; i += blockDim.x) {
    const double v = acc ? d.xchg_cand[i] : d.xcam_loc[i];
    d.xcam_loc[i] = v;
    d.xchg_cam[i] = v;
  }
}

__device__ void decide_step(LmState& s, const double* u, const double* c) {
  if (s.done) return;
  if (u[kUTimeout] > 0.0) {
    // a Cholesky hand-off wait hit its spin limit: the step's solution is not trusted, and the solve reports
    // it (summary.error in the reference, slam.cpp:520) instead of silently rejecting the step
    s.sync_timeouts += (int)u[kUTimeout];
    s.done = 1; s.ok = 0; s.termination = SG_DEVICE_TIMEOUT;
    return;
  }
  const double model = u[kUModel] + c[kCModel];
  const double step2 = u[kUStep2] + c[kCStep2];
  const bool solved = u[kULinFail] == 0.0 && c[kCFail] == 0.0 && isfinite(step2) && isfinite(model);
  const bool valid = solved && !(model < 0.0);
  bool success = false;
  s.last_model = model;
  if (!valid) {
    s.n_invalid += 1;
    s.consecutive_invalid += 1;
    if (!s.disable_term && s.consecutive_invalid >= s.max_invalid) {
      s.done = 1; s.ok = 0; s.termination = SG_NUMERICAL_FAILURE;
      return;
    }
  } else {
    s.consecutive_invalid = 0;
    const double new_cost = u[kUCandFail] > 0.0 ? DBL_MAX : u[kUCandCost] + c[kCCandCost];
    const double step_norm = sqrt(step2);
    s.last_new_cost = new_cost;
    s.last_step_norm = step_norm;
    if (!s.disable_term && step_norm <= s.ptol * (s.x_norm + s.ptol)) {
      s.done = 1; s.ok = 1; s.termination = SG_PARAMETER_TOLERANCE;
      return;
    }
    const double cost_change = s.cost - new_cost;
    if (!s.disable_term && fabs(cost_change) < s.ftol * s.cost) {
      s.done = 1; s.ok = 1; s.termination = SG_FUNCTION_TOLERANCE;
      return;
    }
    const double rel = cost_change / model;
    s.last_rel_decrease = rel;
    success = rel > s.min_rel_dec;
    if (success) {
      s.n_succ += 1;
      const double t = 2.0 * rel - 1.0;
      s.radius = s.radius / fmax(1.0 / 3.0, 1.0 - t * t * t);
      s.radius = fmin(s.max_radius, s.radius);
      s.decrease_factor = 2.0;
      s.reuse_diag = 0;
      s.cur ^= 1;
      s.accepted = 1;
      s.x_norm = sqrt(u[kUCandX2] + c[kCCandX2]);
      s.cost = new_cost;
      s.need_lin = 1;   // the iteration is pushed after the gradient test in k_cam_finalize
      return;
    }
  }
  // rejected (StepRejected) or invalid (StepIsInvalid == StepRejected(0))
  if (valid) s.n_unsucc += 1;
  else s.n_unsucc += 1;
  s.radius = s.radius / s.decrease_factor;
  s.decrease_factor *= 2.0;
  s.reuse_diag = 1;
  if (!s.disable_term && s.radius < s.min_radius) {
    s.done = 1; s.ok = 1; s.termination = SG_PARAMETER_TOLERANCE;
    return;
  }
  if (s.always_lin) {
    // benchmark unit (every LM iteration linearizes): re-linearize at the same x — the same
    // residuals, Jacobians and diagonal, so the same trajectory — and let k_cam_finalize push the iteration
    s.need_lin = 1;
    return;
  }
  s.pushed += 1;
  s.min_pushed_cost = fmin(s.min_pushed_cost, s.cost);
}

// Zero the S accumulation target before k_S_reduce writes the new system (upper blocks only are
// rewritten; the lower part is never read).
__global__ void k_evaluate(Dev d, double* resid, double* cost_out, int32_t* nfail) {
  // residual sweep at x[cur] (parity / ReprojectionError check), observation order = device order
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= d.M) return;
  const int cur = d.st->cur & 1;
  // find the point of o: binary search in poff
  int lo = 0, hi = d.P;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (d.poff[mid] <= o) lo = mid;
    else hi = mid;
  }
  const int p = lo, f = d.obs_frame[o];
  double uv[2];
  if (!Project(d.q[cur] + 4 * f, d.t[cur] + 3 * f, d.k[cur] + 7 * d.frame_cam[f], d.X[cur] + 4 * p, uv)) {
    resid[2 * o] = 0.0;
    resid[2 * o + 1] = 0.0;
    atomicAdd(nfail, 1);
    return;
  }
  const double e0 = uv[0] - d.obs_pt[2 * o], e1 = uv[1] - d.obs_pt[2 * o + 1];
  resid[2 * o] = e0;
  resid[2 * o + 1] = e1;
  if (!d.obs_fixed[o]) {
    double rho0, rho1;
    Cauchy(e0 * e0 + e1 * e1, d.b, d.inv_b, &rho0, &rho1);
    atomicAdd(cost_out, 0.5 * rho0);
  }
}

// ------------------------------------------------------------------------------------------------
// ReprojectMap (slam.cpp:523-548): every observation of the map, disabled ones included.
__global__ __launch_bounds__(256) void k_reproject_map(const double* k, const double* q, const double* t,
                                                        const int32_t* frame_cam, const double* X,
                                                        const double* pt, const int32_t* of,
                                                        const int32_t* op, int M, double* err,
                                                        double* partial) {
  __shared__ double red[4];
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  double nrm = 0.0, cnt = 0.0;
  if (o < M) {
    const int f = of[o], p = op[o];
    double uv[2];
    const double px = pt[2 * o], py = pt[2 * o + 1];
    if (Project(q + 4 * f, t + 3 * f, k + 7 * frame_cam[f], X + 4 * p, uv)) {
      const double e0 = uv[0] - px, e1 = uv[1] - py;
      err[2 * o] = e0;
      err[2 * o + 1] = e1;
      nrm = sqrt(e0 * e0 + e1 * e1);
      cnt = 1.0;
    } else {
      err[2 * o] = px;   // o->error = o->pt, left as is when the projection fails (slam.cpp:529,539-541)
      err[2 * o + 1] = py;
    }
  }
  nrm = block_sum<256>(nrm, red);
  cnt = block_sum<256>(cnt, red);
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = nrm;
    partial[2 * blockIdx.x + 1] = cnt;
  }
}
__global__ __launch_bounds__(64) void k_reproject_reduce(const double* partial, int nb, double* out) {
  double s = 0.0, c = 0.0;
  for (int i = threadIdx.x; i < nb; i += 64) {
    s += partial[2 * i];
    c += partial[2 * i + 1];
  }
  s = wave_sum(s);
  c = wave_sum(c);
  if (threadIdx.x == 0) {
    out[0] = c > 0.0 ? s / c : 0.0;
    out[1] = c;
  }
}

// ================================================================================================
// Host driver

enum KernelId { kKLin = 0, kKCamReduce, kKCamFinal, kKSchur, kKSReduce, kKChol, kKPointUpd, kKUpdRed, kKDecide,
                kKXchg, kKNum };
static const char* kKernelNames[kKNum] = {"linearize", "cam_reduce", "cam_finalize", "schur", "S_reduce",
                                          "cholesky", "point_update", "upd_reduce", "decide", "exchange"};

// The tiled Cholesky's instantiations (kLa bit 0 look-ahead, bit 1 readlane factor, bit 2 Dinv, bit 3 register
// / MFMA factor; SG_CHOL_LOOKAHEAD / SG_CHOL_FACTOR (1 readlane, 2 MFMA) / SG_CHOL_DINV): [0] the stamped build of
// the default, then the variants in kCholTilesLa's order.
static constexpr int kCholTilesLa[] = {0, 1, 3, 5, 8, 9, 17};
static const void* const kCholTilesStamped[] = {(const void*)k_chol_tiles<true, 1>, (const void*)k_chol_tiles<true, 9>,
                                                (const void*)k_chol_tiles<true, 17>};
static const void* const kCholTilesKernels[] = {
    (const void*)k_chol_tiles<true, 1>, (const void*)k_chol_tiles<false, 0>, (const void*)k_chol_tiles<false, 1>,
    (const void*)k_chol_tiles<false, 3>, (const void*)k_chol_tiles<false, 5>, (const void*)k_chol_tiles<false, 8>,
    (const void*)k_chol_tiles<false, 9>, (const void*)k_chol_tiles<false, 17>};

// The SG_CHOL_* variant flags as k_chol_tiles' kLa, and its index in kCholTilesLa (-1: not instantiated).
int BaSolver::CholTilesLa() const {
  return (chol_lookahead_ ? 1 : 0) | (chol_factor_ == 1 ? 2 : 0) | (chol_dinv_ ? 4 : 0) | (chol_factor_ == 2 ? 8 : 0) |
         (chol_dataflow_ ? 16 : 0);
}
static int chol_tiles_index(int la) {
  for (int i = 0; i < (int)(sizeof(kCholTilesLa) / sizeof(int)); ++i)
    if (kCholTilesLa[i] == la) return i;
  return -1;
}
// stamped builds exist for the default (look-ahead), the MFMA factor and the dataflow sync only
static bool chol_tiles_stamped(int la) { return la == 1 || la == 9 || la == 17; }

void BaSolver::LaunchCholTiles(bool stamp, int la, dim3 grid, const Dev& d, int flags) {
  const int idx = chol_tiles_index(la);   // validated in the constructor (CheckCholVariant)
  const void* f = stamp ? kCholTilesStamped[(la & 16) ? 2 : (la & 8) ? 1 : 0] : kCholTilesKernels[1 + idx];
  Dev dd = d;
  // bordered: the frame band ends follow the arrowhead's panel ends in work_i_
  const int32_t* pj = (const int32_t*)work_i_.ptr + (chol_border_ ? (n_ + kCholNb - 1) / kCholNb : 0);
  double* wg = Wg_.ptr;
  int32_t* tf = tflag_.ptr;
  int nd = chol_nd_;
  if (chol_border_) flags |= 8;
  void* args[] = {&dd, &pj, &wg, &tf, &nd, &flags};
  SG_HIP_CHECK(hipLaunchKernel(f, grid, dim3(kTileThreads), args, tile_lds_, stream_));
  if (chol_border_) {
    const int ntf = (6 * NB_ + kCholNb - 1) / kCholNb;
    hipLaunchKernelGGL((border_flags_ & 1) ? k_chol_border<true> : k_chol_border<false>, dim3(1), dim3(kBordThreads),
                       border_lds_doubles(ntf, border_flags_, F_, D_, n_) * sizeof(double), stream_, d, Wg_.ptr,
                       border_flags_);
  }
}

BaSolver::BaSolver(const sg_device_options& dev) : dev_(dev) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) throw Error(SG_ENODEV, "no HIP device available");
  SG_REQUIRE(dev.device >= 0 && dev.device < ndev, SG_ENODEV, "device ordinal out of range");
  SG_REQUIRE(dev.precision == 0, SG_EINVAL,
             "sg_device_options.precision: only 0 (fp64, the reference's arithmetic) is implemented");
  SG_HIP_CHECK(hipSetDevice(dev.device));
  SG_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  // the side stream only in the Schur-overlap mode: every stream holds a hardware queue (GPU_MAX_HW_QUEUES = 4
  // per process on the pool), and an idle queue that has to be scheduled again was the one measured cause of
  // the replay's late load starts (tools/e2e_replay.py)
  if (overlap_ok_) SG_HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  SG_HIP_CHECK(hipEventCreateWithFlags(&ev_lin_, hipEventDisableTiming));
  SG_HIP_CHECK(hipEventCreateWithFlags(&ev_schur_, hipEventDisableTiming));
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev.device) == hipSuccess && prop.multiProcessorCount > 0)
      ncu_ = prop.multiProcessorCount;
  }
  // the SG_CHOL_* / SG_STAMP development switches are fixed per process: refuse a combination without a build
  // here, not in the middle of a solve (and never launch a stamped build of a different variant)
  {
    const int la = CholTilesLa();
    SG_REQUIRE(chol_tiles_index(la) >= 0, SG_EINVAL,
               "this combination of SG_CHOL_* variants is not instantiated (SG_CHOL_LOOKAHEAD=0 runs alone)");
    const bool stamp = getenv("SG_STAMP") && getenv("SG_STAMP")[0] == '1';
    SG_REQUIRE(!stamp || chol_tiles_stamped(la), SG_EINVAL,
               "SG_STAMP=1 has no stamped build of this SG_CHOL_* variant (the default, SG_CHOL_FACTOR=2 and "
               "SG_CHOL_DATAFLOW=1 have one)");
  }
  stager_.reset(new Stager());
  SG_HIP_CHECK(hipFuncSetAttribute((const void*)k_cholesky_window<false>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCholLds));
  SG_HIP_CHECK(hipFuncSetAttribute((const void*)k_cholesky_window<true>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCholLds));
  {
    // k_chol_tiles' dynamic LDS (x, z', band ends, staged candidate operands) grows with the map: grant the
    // most the CU allows beside the kernel's static LDS once, here, so a load never changes the attribute
    size_t lim = 160 * 1024;
    for (const void* f : kCholTilesKernels) {
      hipFuncAttributes fa;
      SG_HIP_CHECK(hipFuncGetAttributes(&fa, f));
      lim = std::min(lim, (size_t)160 * 1024 - fa.sharedSizeBytes);
    }
    for (const void* f : kCholTilesKernels)
      SG_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lim));
    for (const void* f : kCholTilesStamped)
      SG_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lim));
    tile_lds_set_ = lim;
    hipFuncAttributes ga;
    SG_HIP_CHECK(hipFuncGetAttributes(&ga, (const void*)k_cholesky_global<true>));
    gchol_lds_max_ = (size_t)160 * 1024 - ga.sharedSizeBytes;
    for (const void* f : {(const void*)k_cholesky_global<true>, (const void*)k_cholesky_global<false>})
      SG_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)gchol_lds_max_));
    border_lds_max_ = (size_t)160 * 1024;
    for (const void* f : {(const void*)k_chol_border<true>, (const void*)k_chol_border<false>}) {
      hipFuncAttributes ba;
      SG_HIP_CHECK(hipFuncGetAttributes(&ba, f));
      border_lds_max_ = std::min(border_lds_max_, (size_t)160 * 1024 - ba.sharedSizeBytes);
    }
    SG_REQUIRE(border_lds_doubles(kTileMaxNT, 0, 0, 0, 0) * sizeof(double) <= border_lds_max_, SG_EINVAL,
               "k_chol_border: LDS for kTileMaxNT rows");
    for (const void* f : {(const void*)k_chol_border<true>, (const void*)k_chol_border<false>})
      SG_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)border_lds_max_));
  }
  st_.Resize(1);
  timers_.resize(kKNum);
  for (int i = 0; i < kKNum; ++i) timers_[i].name = kKernelNames[i];
}

BaSolver::~BaSolver() {
  DropGraph();
  for (auto& t : timers_)
    for (auto e : t.ev) (void)hipEventDestroy(e);
  if (ev_wait_) (void)hipEventDestroy(ev_wait_);
  if (ev_idle_) (void)hipEventDestroy(ev_idle_);
  if (ev_idle_prev_) (void)hipEventDestroy(ev_idle_prev_);
  if (ev_lin_) (void)hipEventDestroy(ev_lin_);
  if (ev_schur_) (void)hipEventDestroy(ev_schur_);
  if (side_) (void)hipStreamDestroy(side_);
  if (stream_) (void)hipStreamDestroy(stream_);
}

void BaSolver::UniqueId(void* id128) { RcclComm::UniqueId(id128); }

void BaSolver::CommInit(const void* id128, int nranks, int rank) {
  SG_REQUIRE(!loaded_, SG_EINVAL, "sg_ba_comm_init must precede sg_ba_load (exchange buffers are sized by it)");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  comm_.reset(new RcclComm(id128, nranks, rank));
  dev_.nranks = nranks;
  dev_.rank = rank;
}

void BaSolver::CommInitLocal(std::shared_ptr<LocalGroup> g, int rank) {
  SG_REQUIRE(!loaded_, SG_EINVAL, "sg_ba_comm_init_local must precede sg_ba_load");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  comm_.reset(new LocalComm(std::move(g), rank));
  dev_.nranks = comm_->nranks();
  dev_.rank = rank;
}

void BaSolver::CommInitHost(int nranks, int rank, int (*fn)(double*, long long, int, void*), void* user) {
  SG_REQUIRE(!loaded_, SG_EINVAL, "sg_ba_comm_init_host must precede sg_ba_load");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  comm_.reset(new HostComm(nranks, rank, fn, user));
  dev_.nranks = comm_->nranks();
  dev_.rank = rank;
}

int BaSolver::nranks() const { return comm_ ? comm_->nranks() : 1; }

void BaSolver::AllReduceSum(double* buf, size_t n) {
  if (comm_ && (comm_->nranks() > 1 || comm_force_)) {
    comm_->AllReduceSum(buf, n, stream_);
    ++nallreduce_;
  }
}

__global__ __launch_bounds__(256) void k_fill_obs_pnt(const int32_t* __restrict__ poff, int32_t* __restrict__ obs_pnt,
                                                      int P) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  for (int o = poff[i]; o < poff[i + 1]; ++o) obs_pnt[o] = i;
}

void BaSolver::Load(const sg_problem& p) {
  DropGraph();   // the captured iteration holds this load's device pointers and sizes
  static const bool host_timing = getenv("SG_HOST_TIMING") != nullptr;   // development aid: phase times
  auto lt0 = std::chrono::steady_clock::now();
  std::string lap_log;
  auto lap = [&](const char* what) {
    if (!host_timing) return;
    const auto t = std::chrono::steady_clock::now();
    char buf[96];
    snprintf(buf, sizeof(buf), " %s %.2f", what, std::chrono::duration<double, std::milli>(t - lt0).count());
    lap_log += buf;
    lt0 = t;
  };
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  // a device mark at the load's start, with its host time: the GPU time from here to the last mark against the
  // host's wall time tells a late device (its queue started late) from a late host (the waiting thread)
  auto load_t0 = std::chrono::steady_clock::now();
  const bool idle_valid_prev = idle_valid_;
  const double idle_gap_host =
      idle_valid_ ? std::chrono::duration<double, std::milli>(load_t0 - idle_host_).count() : 0.0;
  std::swap(ev_idle_, ev_idle_prev_);   // (this load's own waits re-mark ev_idle_)
  if (host_timing) DevMark(stream_, 4);
  {
    // Everything that can reject this rank's problem runs before the first collective, and the verdict rides
    // in that collective (2: some rank's problem is invalid), so that all ranks fail together instead of
    // leaving the others blocked in an all-reduce.
    int vcode = SG_OK;
    std::string verr;
    try {
      ValidateProblem(&p);
      SG_REQUIRE(!p.cameras_free || (p.num_cameras <= kMaxIntrCams && nranks() == 1), SG_EINVAL,
                 "free intrinsics: at most 4 cameras, on one rank (landmark shards keep the intrinsics constant)");
      SG_REQUIRE(p.num_cameras <= 0xff, SG_EINVAL, "too many cameras for the device solver");
      int nfree = 0;
      for (int f = 0; f < p.num_frames; ++f) nfree += (p.frame_rot_free[f] || p.frame_trans_free[f]) ? 1 : 0;
      SG_REQUIRE(nfree < 0xffff, SG_EINVAL, "too many free frames for the device solver");
      std::vector<int32_t> cnt(p.num_points, 0);
      for (int o = 0; o < p.num_obs; ++o)
        SG_REQUIRE(++cnt[p.obs_point[o]] < 65536, SG_EINVAL, "a point has 65536 or more observations");
    } catch (const Error& e) {
      vcode = e.code;
      verr = e.what();
    }
    // incremental update: every rank must take the same path (the full path has a load-time all-reduce)
    double changed = vcode != SG_OK ? 2.0 : (loaded_ && !getenv("SG_NO_REUSE") && SameStructure(p)) ? 0.0 : 1.0;
    if (comm_ && (comm_->nranks() > 1 || comm_force_)) {
      DBuf<double> flag;
      flag.Upload(std::vector<double>{changed}, stream_);
      comm_->AllReduceMax(flag.ptr, 1, stream_);
      SG_HIP_CHECK(hipMemcpyAsync(&changed, flag.ptr, sizeof(double), hipMemcpyDeviceToHost, stream_));
      SG_HIP_CHECK(hipStreamSynchronize(stream_));
    }
    if (vcode != SG_OK) throw Error(vcode, verr);
    if (changed == 2.0) throw Error(SG_EINVAL, "another landmark shard's problem failed validation");
    if (changed == 0.0) {
      LoadValues(p);
      lap("values");
      if (host_timing) fprintf(stderr, "[sg] Load phases (ms):%s\n", lap_log.c_str());
      return;
    }
  }
  // Full path: the structure and every device list are rebuilt below.  Until that completes, this solver
  // holds no usable problem: a failure part way (a device allocation, a hipFuncSetAttribute) must not leave
  // the previous problem's structure key matching a later load's value-only path.
  loaded_ = false;
  began_ = false;
  skey_ = StructKey{};
  stager_->Clear();
  F_ = p.num_frames;
  P_ = p.num_points;
  M_ = p.num_obs;
  D_ = p.num_dist;
  ncam_ = p.num_cameras;
  range_b_ = p.range * p.range;
  fd_target_ = p.dist_target;
  fd_b2_ = p.dist_range * p.dist_range;
  // camera blocks: every frame with a free rotation or translation
  std::vector<int32_t> frame_block(F_, -1);
  NB_ = 0;
  for (int f = 0; f < F_; ++f)
    if (p.frame_rot_free[f] || p.frame_trans_free[f]) frame_block[f] = NB_++;
  nk_ = p.cameras_free ? 7 * ncam_ : 0;
  n_ = 6 * NB_ + nk_;   // frame columns, then the free intrinsics
  stab_b_ = p.stab_range * p.stab_range;
  lap("blocks");
  // point order: by first free block (points without free-frame observations last)
  std::vector<int32_t> pfirst(P_, NB_), plast(P_, -1), pcount(P_, 0);
  for (int o = 0; o < M_; ++o) {
    const int pt = p.obs_point[o], b = frame_block[p.obs_frame[o]];
    pcount[pt]++;
    if (b >= 0) {
      pfirst[pt] = std::min(pfirst[pt], b);
      plast[pt] = std::max(plast[pt], b);
    }
  }
  // stable counting sort on the key pfirst in [0, NB]
  point_perm_.resize(P_);
  std::vector<int32_t> inv_perm(P_);
  {
    std::vector<int32_t> bstart(NB_ + 2, 0);
    for (int i = 0; i < P_; ++i) bstart[pfirst[i] + 1]++;
    for (int b = 0; b <= NB_; ++b) bstart[b + 1] += bstart[b];
    for (int i = 0; i < P_; ++i) {
      const int pos = bstart[pfirst[i]]++;
      point_perm_[pos] = i;
      inv_perm[i] = pos;
    }
  }
  lap("point-order");
  // observations: CSR by device point order (stable in problem order)
  std::vector<int32_t> poff(P_ + 1, 0);
  for (int o = 0; o < M_; ++o) poff[inv_perm[p.obs_point[o]] + 1]++;
  for (int i = 0; i < P_; ++i) poff[i + 1] += poff[i];
  obs_perm_.assign(M_, 0);
  {
    std::vector<int32_t> fill(poff.begin(), poff.end() - 1);
    for (int o = 0; o < M_; ++o) obs_perm_[fill[inv_perm[p.obs_point[o]]]++] = o;
    // within a point: observations of constant frames first, then by camera block (stable), so that a point
    // observed once in every block of its span finds the observation of block b at a fixed offset (k_schur)
    // (a stable insertion sort: a point has a handful of observations, and std::stable_sort allocates a
    // buffer per call)
    if (!getenv("SG_NO_OBS_SORT"))
      for (int i = 0; i < P_; ++i) {
        int32_t* v = obs_perm_.data() + poff[i];
        const int k = poff[i + 1] - poff[i];
        if (k > 64) {
          std::stable_sort(v, v + k, [&](int a, int b) {
            return frame_block[p.obs_frame[a]] < frame_block[p.obs_frame[b]];
          });
          continue;
        }
        for (int x = 1; x < k; ++x) {
          const int32_t o = v[x];
          const int key = frame_block[p.obs_frame[o]];
          int y = x - 1;
          while (y >= 0 && frame_block[p.obs_frame[v[y]]] > key) {
            v[y + 1] = v[y];
            --y;
          }
          v[y + 1] = o;
        }
      }
  }
  std::vector<double> obs_pt(2 * (size_t)M_);
  std::vector<int32_t> obs_frame(M_);
  std::vector<uint8_t> obs_fixed(M_), pfree(P_);
  std::vector<double> X(4 * (size_t)P_);
  for (int i = 0; i < P_; ++i) {
    const int pt = point_perm_[i];
    pfree[i] = p.point_free[pt];
    for (int a = 0; a < 4; ++a) X[4 * i + a] = p.X[4 * pt + a];
  }
  std::vector<int32_t> obs_meta(M_);
  {
    // per frame: the frame part of the packed observation word
    std::vector<int32_t> fmeta(F_);
    for (int f = 0; f < F_; ++f)
      fmeta[f] = (frame_block[f] + 1) | (p.frame_camera[f] << kMetaCamShift) | (p.frame_rot_free[f] ? kMetaRot : 0) |
                 (p.frame_trans_free[f] ? kMetaTrans : 0);
    for (int o = 0; o < M_; ++o) {
      const int src = obs_perm_[o], f = p.obs_frame[src];
      const bool pf = p.point_free[p.obs_point[src]] != 0;
      obs_pt[2 * o] = p.obs_pt[2 * src];
      obs_pt[2 * o + 1] = p.obs_pt[2 * src + 1];
      obs_frame[o] = f;
      obs_fixed[o] = frame_block[f] < 0 && !pf && !p.cameras_free;
      obs_meta[o] = fmeta[f] | (pf ? kMetaPfree : 0) | (obs_fixed[o] ? kMetaFixed : 0);
    }
  }
  lap("obs-csr");
  // upload batch 1 — poses, intrinsics, points (current slot; the candidate slot is a device copy) and the
  // observation arrays: its pinned copy and DMA overlap the host's work-list construction below (stager.h)
  hipStream_t s = stream_;
  Stager& stg = *stager_;
  stg.ResetBytes();
  stg.AddInto(k_, std::max<size_t>(14 * (size_t)ncam_, 1),
              ncam_ > 0 ? std::vector<double>(p.k, p.k + 7 * ncam_) : std::vector<double>{0.0});
  stg.AddInto(q_, 8 * (size_t)F_, std::vector<double>(p.q, p.q + 4 * F_));
  stg.AddInto(t_, 6 * (size_t)F_, std::vector<double>(p.t, p.t + 3 * F_));
  stg.AddInto(X_, 8 * (size_t)P_, X);
  stg.Add(frame_cam_, std::vector<int32_t>(p.frame_camera, p.frame_camera + F_));
  stg.Add(frame_block_, frame_block);
  stg.Add(rot_free_, std::vector<uint8_t>(p.frame_rot_free, p.frame_rot_free + F_));
  stg.Add(trans_free_, std::vector<uint8_t>(p.frame_trans_free, p.frame_trans_free + F_));
  stg.Add(pfree_, pfree);
  stg.Add(poff_, poff);
  stg.Add(obs_pt_, obs_pt);
  stg.Add(obs_frame_, obs_frame);
  stg.Add(obs_fixed_, obs_fixed);
  stg.Add(obs_meta_, obs_meta.empty() ? std::vector<int32_t>{0} : obs_meta);
  if (host_timing) DevMark(s, 0);
  stg.Flush(s);
  {
    auto dup = [&](double* base, size_t half) {   // candidate slot = current slot
      if (half)   // a kernel, not a copy-engine hipMemcpyAsync (see hostmirror.h)
        hipLaunchKernelGGL(k_copy_u64, dim3((unsigned)std::min<size_t>(256, (half + 255) / 256)), dim3(256), 0, s,
                           reinterpret_cast<const unsigned long long*>(base),
                           reinterpret_cast<unsigned long long*>(base + half), half);
    };
    dup(k_.ptr, 7 * (size_t)ncam_);
    dup(q_.ptr, 4 * (size_t)F_);
    dup(t_.ptr, 3 * (size_t)F_);
    dup(X_.ptr, 4 * (size_t)P_);
    // the point of every observation (device order) from the CSR, on the device
    obs_pnt_.Resize(std::max(M_, 1));
    if (P_ > 0)
      hipLaunchKernelGGL(k_fill_obs_pnt, dim3((P_ + 255) / 256), dim3(256), 0, s, (const int32_t*)poff_.ptr,
                         obs_pnt_.ptr, P_);
    SG_HIP_CHECK(hipGetLastError());
  }
  lap("upload-1");
  // Schur work lists (see SchurSeg): the cells of every free point (one per block of its span, with the
  // point's observations in that block), segments of consecutive points whose columns fit kSchurTW tiles of
  // S, their batches, and each wide point's observation pairs (s <= t, both on free frames).
  std::vector<int32_t> pinfo(2 * (size_t)std::max(P_, 1), 0), pmx(4 * (size_t)std::max(P_, 1), 0), cells, cell_obs;
  std::vector<SchurSeg> segs;
  std::vector<SchurBatch> sbatch;
  std::vector<WideSeg> wsegs;
  std::vector<int32_t> pairs_flat;   // int2 per pair (wide points)
  int s_off = 0;
  // k_linearize decomposition (see LinChunk): rounds of whole points (<= kLinObs observations), up to
  // maxr rounds per chunk sharing one camera window; fewer rounds per chunk on small problems so that the
  // grid still fills the chip.
  std::vector<LinRound> lrounds;
  std::vector<LinChunk> lchunks;
  std::vector<uint16_t> llist;
  llist.reserve((size_t)M_ + (size_t)M_ / 4 + 64);
  int lcam_off = 0;
  std::vector<int> cnt;   // per round: window-block counters (scratch, reused)
  {
    int maxr = std::max(1, std::min(kLinMaxRounds, M_ / (kLinObs * 1024)));
    if (getenv("SG_LIN_MAXR")) maxr = std::max(1, atoi(getenv("SG_LIN_MAXR")));   // tuning experiments
    auto kobs = [&](int i) { return poff[i + 1] - poff[i]; };
    auto constonly = [&](int i) { return pfirst[point_perm_[i]] >= NB_; };
    auto pspan = [&](int i) { return constonly(i) ? 0 : plast[point_perm_[i]] - pfirst[point_perm_[i]] + 1; };
    for (int i = 0; i < P_;) {
      LinChunk c{};
      c.p0 = i;
      c.r0 = (int)lrounds.size();
      if (kobs(i) > kLinObs || pspan(i) > kLinNbMax) {
        c.wide = 1;
        for (int o = poff[i]; o < poff[i + 1]; o += kLinObs)
          lrounds.push_back(LinRound{o, std::min(o + kLinObs, poff[i + 1]), i, i + 1, 0, 0});
        c.p1 = ++i;
      } else {
        const bool co = constonly(i);
        int lo = co ? 0 : pfirst[point_perm_[i]], hi = co ? -1 : plast[point_perm_[i]];
        int j = i, nr = 0;
        LinRound R{poff[i], poff[i], i, i, 0, 0};
        while (j < P_) {
          if (kobs(j) > kLinObs || pspan(j) > kLinNbMax || constonly(j) != co) break;
          int l2 = lo, h2 = hi;
          if (!co) {
            l2 = std::min(lo, pfirst[point_perm_[j]]);
            h2 = std::max(hi, plast[point_perm_[j]]);
            if (h2 - l2 + 1 > kLinNbMax) break;
          }
          if (R.o1 - R.o0 + kobs(j) > kLinObs || R.p1 - R.p0 >= kLinPts) {
            if (nr + 1 >= maxr) break;
            lrounds.push_back(R);
            ++nr;
            R = LinRound{poff[j], poff[j], j, j, 0, 0};
          }
          R.o1 += kobs(j);
          R.p1 = j + 1;
          lo = l2;
          hi = h2;
          ++j;
        }
        lrounds.push_back(R);
        c.p1 = j;
        c.b_lo = lo;
        c.nb = co ? 0 : hi - lo + 1;
        i = j;
      }
      c.r1 = (int)lrounds.size();
      c.cam_off = lcam_off;
      lcam_off += c.nb * kCamV;
      // per round: the window-block offsets and the round-local observation indices sorted by block
      for (int r = c.r0; r < c.r1; ++r) {
        LinRound& R = lrounds[r];
        R.lst = (int)llist.size();
        if (c.nb == 0) continue;
        cnt.assign(c.nb + 1, 0);
        for (int o = R.o0; o < R.o1; ++o) {
          const int b = frame_block[obs_frame[o]];
          if (b >= 0) cnt[b - c.b_lo + 1]++;
        }
        for (int k = 0; k < c.nb; ++k) cnt[k + 1] += cnt[k];
        const size_t base = llist.size();
        llist.resize(base + c.nb + 1 + cnt[c.nb]);
        for (int k = 0; k <= c.nb; ++k) llist[base + k] = (uint16_t)cnt[k];
        for (int o = R.o0; o < R.o1; ++o) {
          const int b = frame_block[obs_frame[o]];
          if (b >= 0) llist[base + c.nb + 1 + cnt[b - c.b_lo]++] = (uint16_t)(o - R.o0);
        }
      }
      lchunks.push_back(c);
    }
  }
  nlin_ = (int)lchunks.size();
  // two waves per chunk (its rounds split between them) while the doubled grid still fits the chip at three
  // waves per SIMD (k_linearize's occupancy): config 2's ~1.5 k chunks; one wave per chunk when there are more
  // chunks than that (config 5, the scaled sweep), where the second wave only adds the combine
  lin_waves_ = 2 * (long long)nlin_ <= 12LL * ncu_ ? 2 : 1;
  if (const char* e = getenv("SG_LIN_WAVES")) lin_waves_ = atoi(e) == 2 ? 2 : 1;   // A/B and tests
  std::vector<int32_t> pu_units;   // k_point_update work units: a round index, or -(chunk + 1) for wide chunks
  for (int c = 0; c < nlin_; ++c) {
    lchunks[c].u0 = (int)pu_units.size();   // k_update_lin writes the units' scalars
    if (lchunks[c].wide)
      pu_units.push_back(-(c + 1));
    else
      for (int r = lchunks[c].r0; r < lchunks[c].r1; ++r) pu_units.push_back(r);
  }
  npu_ = (int)pu_units.size();
  if (pu_units.empty()) pu_units.push_back(0);
  lap("lin-lists");
  std::vector<int32_t> obs_blk(M_);
  for (int o = 0; o < M_; ++o) obs_blk[o] = frame_block[obs_frame[o]];
  // span in blocks of a free point's Schur terms (0: none)
  auto sspan = [&](int i) {
    const int pt = point_perm_[i];
    return (pfree[i] && pfirst[pt] < NB_) ? plast[pt] - pfirst[pt] + 1 : 0;
  };
  std::vector<int32_t> simple_obs(std::max(P_, 1), -1);   // observation of the first block if one per block
  int ncell = 0;
  npairs_ = 0;
  schur_mfma_ = 0.0;
  {
    std::vector<std::pair<int, int>> bo;
    cells.reserve(4 * (size_t)M_ + 4);
    cell_obs.reserve((size_t)M_ / 4 + 1);
    for (int i = 0; i < P_; ++i) {
      size_t kb = 0;
      for (int o = poff[i]; o < poff[i + 1]; ++o) kb += obs_blk[o] >= 0;
      if (pfree[i]) npairs_ += kb * (kb + 1) / 2;
      const int sp = sspan(i);
      if (sp == 0 || sp > kSegNbMax) continue;
      const int pf = pfirst[point_perm_[i]];
      pinfo[2 * i] = (int)(cells.size() / 4);
      pinfo[2 * i + 1] = (pf << 8) | sp;
      bo.clear();
      for (int o = poff[i]; o < poff[i + 1]; ++o)
        if (obs_blk[o] >= 0) bo.emplace_back(obs_blk[o], o);
      if (!std::is_sorted(bo.begin(), bo.end())) std::sort(bo.begin(), bo.end());   // sorted at load already
      {
        bool one = (int)bo.size() == sp;   // observations sorted by block at load: consecutive
        for (int q = 0; one && q < sp; ++q) one = bo[q].first == pf + q && bo[q].second == bo[0].second + q;
        if (one) simple_obs[i] = bo[0].second;
      }
      size_t k = 0;
      for (int b = pf; b < pf + sp; ++b) {
        // {first observation or -1, point, (block << 16) | further observations, their offset in cell_obs}
        int o0 = -1;
        if (k < bo.size() && bo[k].first == b) o0 = bo[k++].second;
        const int k1 = (int)cell_obs.size();
        while (k < bo.size() && bo[k].first == b) cell_obs.push_back(bo[k++].second);
        cells.insert(cells.end(), {o0, i, (int)(((unsigned)b << 16) | (unsigned)(cell_obs.size() - k1)), k1});
      }
    }
    ncell = (int)cells.size() / 4;
    if (cells.empty()) cells.assign(4, 0);
    if (cell_obs.empty()) cell_obs.push_back(0);
  }
  {
    // points per segment: one segment per CU (the workgroup's LDS holds one per CU; fewer, longer segments
    // write fewer partial tiles and keep the producer/consumer pipeline full; SG_SCHUR_SEGS: tuning)
    const int ncu = ncu_;
    // (with k_schur beside the camera reduction, one CU per XCD stays free for k_cam_reduce / k_cam_finalize:
    // a k_schur workgroup's 140 KB of LDS leaves no room for them on its CU)
    const int target = getenv("SG_SCHUR_SEGS") ? std::max(1, atoi(getenv("SG_SCHUR_SEGS")))
                                               : (overlap_ok_ ? std::max(1, ncu - 8) : ncu);
    const int maxpts = std::max(16, (P_ + target - 1) / target);
    int cnext = 0;
    for (int i = 0; i < P_;) {
      if (sspan(i) > kSegNbMax) {
        WideSeg w{};
        w.p = i;
        w.pair_lo = (int)pairs_flat.size() / 2;
        for (int os = poff[i]; os < poff[i + 1]; ++os) {
          if (obs_blk[os] < 0) continue;
          for (int ot = os; ot < poff[i + 1]; ++ot) {
            if (obs_blk[ot] < 0) continue;
            pairs_flat.push_back(((os - poff[i]) << 16) | (ot - poff[i]));
            pairs_flat.push_back((obs_blk[os] << 16) | obs_blk[ot]);
          }
        }
        w.pair_hi = (int)pairs_flat.size() / 2;
        wsegs.push_back(w);
        ++i;
        continue;
      }
      SchurSeg sg{};
      sg.p0 = i;
      int clo = INT32_MAX, chi = -1, blo = INT32_MAX, bhi = -1;   // columns [clo, chi), blocks [blo, bhi]
      int j = i;
      while (j < P_ && j - i < maxpts) {
        const int sp = sspan(j);
        if (sp > kSegNbMax) break;
        if (sp > 0) {
          const int pf = pfirst[point_perm_[j]];
          const int l2 = std::min(clo, 6 * pf), h2 = std::max(chi, 6 * (pf + sp));
          if ((h2 + 15) / 16 - l2 / 16 > kSchurTW) break;
          clo = l2;
          chi = h2;
          blo = std::min(blo, pf);
          bhi = std::max(bhi, pf + sp - 1);
        }
        ++j;
      }
      sg.p1 = j;
      if (chi >= 0) {
        sg.t0 = clo / 16;
        sg.ntw = (chi + 15) / 16 - sg.t0;
        sg.b_lo = blo;
        sg.nb = bhi - blo + 1;
      }
      sg.s_off = s_off;
      s_off += sg.ntw * (sg.ntw + 1) / 2 * 256 + 16 * sg.ntw;
      // last window tile of each point's columns (-1: no Schur terms)
      auto pjhi = [&](int k) {
        const int sp = sspan(k);
        return sp == 0 ? -1 : (6 * (pfirst[point_perm_[k]] + sp) - 1 - 16 * sg.t0) / 16;
      };
      sg.bt0 = (int)sbatch.size();
      for (int k = i; k < j;) {
        SchurBatch B{};
        B.p0 = k;
        B.c0 = cnext;
        int nc = 0, nx = 0;
        while (k < j && k - B.p0 < kSchurBatchPts && nx + 64 * (pjhi(k) + 1) <= kSchurXCap &&
               nc + sspan(k) <= 64 * kSchurCellWaves) {
          pmx[4 * k] = nx;
          pmx[4 * k + 1] = pjhi(k);
          pmx[4 * k + 2] = simple_obs[k];
          pmx[4 * k + 3] = nc;
          nx += 64 * (pjhi(k) + 1);
          schur_mfma_ += schur_aug_base(pjhi(k) + 1);
          nc += sspan(k++);
        }
        B.p1 = k;
        B.c1 = B.c0 + nc;
        cnext += nc;
        sbatch.push_back(B);
      }
      sg.bt1 = (int)sbatch.size();
      segs.push_back(sg);
      i = j;
    }
    SG_REQUIRE(cnext == ncell, SG_EINVAL, "Schur cells out of step with the batches");
  }
  nseg_ = (int)segs.size();
  nwide_ = (int)wsegs.size();
  if (pairs_flat.empty()) pairs_flat.assign(2, 0);
  lap("segments");
  // deterministic reduction lists: for every camera block, the slab offsets of the chunk partials that cover
  // it (fixed chunk order), and of the segments' rhs partials
  std::vector<int32_t> cam_loff(NB_ + 1, 0), cam_lidx, r_loff(NB_ + 1, 0), r_lidx;
  {
    std::vector<std::vector<int32_t>> cl(NB_), rl(NB_);
    for (const LinChunk& ch : lchunks) {
      if (ch.wide || ch.nb == 0) continue;
      for (int i = 0; i < ch.nb; ++i) cl[ch.b_lo + i].push_back(ch.cam_off + i * kCamV);
    }
    for (const SchurSeg& sg : segs) {   // rhs partial of block I: window columns 6 I - 16 t0 ..
      const int ntile = sg.ntw * (sg.ntw + 1) / 2;
      for (int i = 0; i < sg.nb; ++i)
        rl[sg.b_lo + i].push_back(sg.s_off + 256 * ntile + 6 * (sg.b_lo + i) - 16 * sg.t0);
    }
    for (int b = 0; b < NB_; ++b) {
      cam_loff[b + 1] = cam_loff[b] + (int)cl[b].size();
      cam_lidx.insert(cam_lidx.end(), cl[b].begin(), cl[b].end());
      r_loff[b + 1] = r_loff[b] + (int)rl[b].size();
      r_lidx.insert(r_lidx.end(), rl[b].begin(), rl[b].end());
    }
    if (cam_lidx.empty()) cam_lidx.push_back(0);
    if (r_lidx.empty()) r_lidx.push_back(0);
  }
  lap("reduce-lists");
  // FrameDistance
  std::vector<int32_t> fd_a(p.dist_frame, p.dist_frame + D_), fd_b(p.dist_prev, p.dist_prev + D_);
  std::vector<int32_t> fd_boff(NB_ + 1, 0), fd_bidx;
  {
    std::vector<std::vector<int32_t>> lists(NB_);
    for (int dd = 0; dd < D_; ++dd) {
      const int ba = frame_block[fd_a[dd]], bb = frame_block[fd_b[dd]];
      if (ba >= 0) lists[ba].push_back(2 * dd);
      if (bb >= 0) lists[bb].push_back(2 * dd + 1);
    }
    for (int b = 0; b < NB_; ++b) {
      fd_boff[b + 1] = fd_boff[b] + (int)lists[b].size();
      fd_bidx.insert(fd_bidx.end(), lists[b].begin(), lists[b].end());
    }
  }
  lap("fd");
  // Cholesky panel envelopes: block column J's first nonzero block row lo(J)
  std::vector<int32_t> lo_blk(NB_);
  for (int b = 0; b < NB_; ++b) lo_blk[b] = b;
  {
    // exact envelope from the observations of each free point (pairs of blocks it couples)
    for (int i = 0; i < P_; ++i) {
      const int pt = point_perm_[i];
      if (pfirst[pt] >= NB_) continue;
      if (!p.point_free[pt]) continue;
      const int lo = pfirst[pt];
      for (int o = poff[i]; o < poff[i + 1]; ++o) {
        const int b = frame_block[obs_frame[o]];
        if (b >= 0) lo_blk[b] = std::min(lo_blk[b], lo);
      }
    }
    for (int dd = 0; dd < D_; ++dd) {
      const int ba = frame_block[fd_a[dd]], bb = frame_block[fd_b[dd]];
      if (ba >= 0 && bb >= 0) {
        const int hi3 = std::max(ba, bb), lo3 = std::min(ba, bb);
        lo_blk[hi3] = std::min(lo_blk[hi3], lo3);
      }
    }
  }
  // Landmark shards: S is summed over every rank's points, so each rank must factor it with the envelope of
  // the whole problem (the union of the shards' envelopes), not of its own points.  One max all-reduce of
  // -lo(J) at load time.
  if (comm_ && (comm_->nranks() > 1 || comm_force_) && NB_ > 0) {
    std::vector<double> neg(NB_);
    for (int b = 0; b < NB_; ++b) neg[b] = -(double)lo_blk[b];
    DBuf<double> env;
    env.Upload(neg, stream_);
    comm_->AllReduceMax(env.ptr, (size_t)NB_, stream_);
    SG_HIP_CHECK(hipMemcpyAsync(neg.data(), env.ptr, NB_ * sizeof(double), hipMemcpyDeviceToHost, stream_));
    SG_HIP_CHECK(hipStreamSynchronize(stream_));
    for (int b = 0; b < NB_; ++b) lo_blk[b] = (int)(-neg[b]);
  }
  const int npanel = (n_ + kCholNb - 1) / kCholNb;
  std::vector<int32_t> panel_jmax(std::max(npanel, 1), 0), panel_bend(std::max(npanel, 1), 0);
  for (int pk = 0; pk < npanel; ++pk) {
    const int row_hi = std::min(n_, (pk + 1) * kCholNb) - 1;   // last row of the panel
    const int blk_hi = row_hi / 6;
    int jmax = (pk + 1) * kCholNb;
    // columns j whose envelope starts at or before the panel's last row block
    for (int b = 0; b < NB_; ++b)
      if (lo_blk[b] <= blk_hi) jmax = std::max(jmax, 6 * b + 6);
    jmax = std::min(jmax, n_);
    panel_jmax[pk] = std::min(n_, (jmax + kCholNb - 1) / kCholNb * kCholNb);   // band end, 16-aligned
    if (nk_) {   // the intrinsics columns couple every frame: S is dense (k_cholesky_global: arrowhead)
      panel_bend[pk] = std::min(jmax, 6 * NB_);
      panel_jmax[pk] = n_;
    }
  }
  if (nk_) panel_jmax.insert(panel_jmax.end(), panel_bend.begin(), panel_bend.end());   // work_i_ tail
  {
    std::vector<int32_t> off(npanel + 1, 0);
    for (int pk = 0; pk < npanel; ++pk)
      off[pk + 1] = off[pk] + std::min(kCholNb, n_ - pk * kCholNb) * (panel_jmax[pk] - pk * kCholNb);
    npack_ = (size_t)off[npanel] + n_;
    stager_->Add(pack_off_, off);
    // + the merged exchange's tail (k_cam_finalize modes 1, 2)
    ntail_ = 2 * (size_t)6 * NB_ + kXNum + nranks() + 1;
    Spk_.Resize(npack_ + ntail_);
  }
  // k_cholesky_global stages each panel's rows in LDS when x and 16 rows of S fit
  // (SG_CHOL_GSTAGE=0: never, so tests reach the unstaged instance at any size)
  chol_gstage_ = (size_t)std::max(n_, 1) * 8 * (1 + kCholNb) <= gchol_lds_max_ &&
                 !(getenv("SG_CHOL_GSTAGE") && atoi(getenv("SG_CHOL_GSTAGE")) == 0);
  chol_window_ = npanel <= kJendSh;   // band ends cached in LDS
  for (int pk = 0; pk < npanel; ++pk)
    if (panel_jmax[pk] - pk * kCholNb > kCholWS) chol_window_ = false;
  band_tiles_ = 0;
  for (int pk = 0; pk < npanel; ++pk)
    band_tiles_ = std::max(band_tiles_, (panel_jmax[pk] + kCholNb - 1) / kCholNb - pk);
  // tiled band Cholesky: every tile row's band within kTB tiles, x and z' of the whole system in LDS
  chol_tiles_ = n_ > 0 && nk_ == 0 && npanel <= kTileMaxNT && !getenv("SG_CHOL_WINDOW");
  for (int pk = 0; pk < npanel; ++pk)
    if ((panel_jmax[pk] + kCholNb - 1) / kCholNb - pk > kTB) chol_tiles_ = false;
  // free intrinsics (one 16-wide border tile): the frame band on k_chol_tiles, the border by k_chol_border
  // (SG_CHOL_BORDER=0: the arrowhead k_cholesky_global)
  chol_border_ = false;
  if (nk_ > 0 && NB_ > 0 && n_ - 6 * NB_ <= kCholNb && !getenv("SG_CHOL_WINDOW") &&
      !(getenv("SG_CHOL_BORDER") && atoi(getenv("SG_CHOL_BORDER")) == 0)) {
    const int ntf = (6 * NB_ + kCholNb - 1) / kCholNb;
    chol_border_ = ntf <= kTileMaxNT;
    for (int pk = 0; pk < ntf; ++pk)
      if ((panel_bend[pk] + kCholNb - 1) / kCholNb - pk > kTB) chol_border_ = false;
    if (chol_border_) {
      chol_tiles_ = true;
      // q_K tiles and the candidate operands in LDS where they fit (else global q_K / chol_candidates)
      border_flags_ = 0;
      for (int f : {1, 2, 3})   // the last that fits: both, else the candidate operands, else the q_K tiles
        if (border_lds_doubles(ntf, f, F_, D_, n_) * sizeof(double) <= border_lds_max_ &&
            (!(f & 2) || (F_ <= kCandMax && D_ <= kCandMax)))
          border_flags_ = f;
    }
  }
  // dissected band: a second workgroup factors the bottom nd tile rows (reversed) while the first factors
  // the top, both meeting at a 7-tile separator (k_chol_tiles); worth it from about 12 tile rows
  chol_nd_ = 0;
  if (chol_tiles_ && !chol_border_ && npanel >= kSplitMinNT &&
      !(getenv("SG_CHOL_SPLIT") && atoi(getenv("SG_CHOL_SPLIT")) == 0))
    chol_nd_ = (npanel - 9) / 2;   // the bottom (nd rows + hand-off) done before the top reaches row m - 1
  if (chol_nd_ > 0 && getenv("SG_CHOL_ND")) chol_nd_ = std::max(1, std::min(atoi(getenv("SG_CHOL_ND")), (npanel - 9) / 2 + 1));
  if (chol_tiles_) {
    // W tiles of the top and bottom halves, the bottom's z' (+ failure slot), the separator contribution
    // and its rhs, then the constants {0, 1}
    std::vector<double> wz((size_t)2 * npanel * kTB * 256 + 16 * (size_t)npanel + 49 * 256 + 7 * 16 + 2, 0.0);
    wz.back() = 1.0;
    stager_->Add(Wg_, wz);
    stager_->Add(tflag_, std::vector<int32_t>(2, 0));
    tile_lds_ = (size_t)npanel * 32 * sizeof(double) + (size_t)(3 * npanel + 1) / 2 * sizeof(double);
    chol_cand_lds_ = !chol_border_ && F_ <= kCandMax && D_ <= kCandMax &&
                     tile_lds_ + CandLds::bytes(F_, D_, n_) <= 100 * 1024 &&
                     tile_lds_ + CandLds::bytes(F_, D_, n_) <= tile_lds_set_;
    if (chol_cand_lds_) tile_lds_ += CandLds::bytes(F_, D_, n_);
    if (tile_lds_ > tile_lds_set_) {   // beyond the LDS granted at construction: the one-workgroup kernels
      chol_tiles_ = false;
      chol_border_ = false;
      chol_nd_ = 0;
    }
  }
  // k_S_reduce work: the band tiles (R <= C) of the frame columns, and per tile the segment tiles covering it
  // (segment order).  A segment tile outside the band is zero (no point couples its rows and columns).
  std::vector<int32_t> stile, s_loff(1, 0), s_lidx;
  {
    const int nft = (6 * NB_ + kCholNb - 1) / kCholNb;
    std::vector<int32_t> row_off(nft + 1, 0), cend(nft, 0);
    for (int R = 0; R < nft; ++R) {
      cend[R] = std::min(nft, (panel_jmax[R] + kCholNb - 1) / kCholNb);
      row_off[R + 1] = row_off[R] + std::max(0, cend[R] - R);
      for (int C = R; C < cend[R]; ++C) stile.push_back((R << 16) | C);
    }
    std::vector<std::vector<int32_t>> tl(stile.size());
    for (const SchurSeg& sg : segs)
      for (int u = 0; u < sg.ntw * (sg.ntw + 1) / 2; ++u) {
        const int R = sg.t0 + schur_tile_r(u), C = sg.t0 + schur_tile_c(u);
        if (R < nft && C < cend[R]) tl[row_off[R] + C - R].push_back(sg.s_off + 256 * u);
      }
    for (const auto& l : tl) {
      s_loff.push_back(s_loff.back() + (int)l.size());
      s_lidx.insert(s_lidx.end(), l.begin(), l.end());
    }
    nstile_ = (int)stile.size();
    if (stile.empty()) stile.push_back(0);
    if (s_lidx.empty()) s_lidx.push_back(0);
  }
  lap("envelope");
  // upload batch 2 — the work lists: one pinned staging copy and one scatter launch (stager.h)
  stg.Add(lchunks_d_, lchunks);
  stg.Add(lrounds_d_, lrounds);
  if (llist.empty()) llist.push_back(0);
  stg.Add(llist_d_, llist);
  stg.Add(segs_, segs.empty() ? std::vector<SchurSeg>(1) : segs);
  stg.Add(sbatch_, sbatch.empty() ? std::vector<SchurBatch>(1) : sbatch);
  stg.Add(wsegs_, wsegs.empty() ? std::vector<WideSeg>(1) : wsegs);
  stg.Add(pinfo_, pinfo);
  stg.Add(pmx_, pmx);
  stg.Add(cells_, cells);
  stg.Add(cell_obs_, cell_obs);
  stg.Add(stile_, stile);
  stg.Add(pairs_, pairs_flat);
  seg_fail_.Resize(std::max(nseg_ + nwide_, 1));
  stg.Add(cam_loff_, cam_loff);
  stg.Add(cam_lidx_, cam_lidx);
  stg.Add(s_loff_, s_loff);
  stg.Add(s_lidx_, s_lidx);
  stg.Add(r_loff_, r_loff);
  stg.Add(r_lidx_, r_lidx);
  // padded to one entry: k_cam_finalize prefetches fd_a[0] / fd_b[0] beside LmState even when D = 0
  stg.Add(fd_a_, fd_a.empty() ? std::vector<int32_t>{0} : fd_a);
  stg.Add(fd_b_, fd_b.empty() ? std::vector<int32_t>{0} : fd_b);
  stg.Add(fd_boff_, fd_boff);
  stg.Add(fd_bidx_, fd_bidx.empty() ? std::vector<int32_t>{0} : fd_bidx);
  stg.Add(work_i_, panel_jmax);
  {
    // FrameDistance cross-block lookup for the on-the-fly assembly: fd_pair[I*NB+J] (I<J) = residual
    std::vector<int32_t> fd_pair((size_t)std::max(NB_, 1) * std::max(NB_, 1), -1);
    for (int dd = 0; dd < D_; ++dd) {
      const int ba = frame_block[fd_a[dd]], bb = frame_block[fd_b[dd]];
      if (ba >= 0 && bb >= 0 && ba != bb) fd_pair[(size_t)std::min(ba, bb) * NB_ + std::max(ba, bb)] = dd;
    }
    stg.Add(fd_pair_, fd_pair);
    rdg_.Resize((size_t)std::max(n_, 1) + kCholNb);   // + padding rows of the last panel
  }
  // the linearization's buffers hold two slots (current point, k_update_lin's candidate)
  jslot_ = (size_t)((std::max(M_, 1) + 63) & ~63) * kJStride;   // whole 64-observation blocks (jidx2)
  J_.Resize(2 * jslot_);
  V_.Resize(2 * 10 * (size_t)std::max(P_, 1));
  g_.Resize(2 * 4 * (size_t)std::max(P_, 1));
  scale_p_.Resize(4 * (size_t)std::max(P_, 1));
  diag_p_.Resize(4 * (size_t)std::max(P_, 1));
  Vinv_.Resize(10 * (size_t)std::max(P_, 1));
  tp_.Resize(4 * (size_t)std::max(P_, 1));
  const size_t nn = std::max(n_, 1);
  scale_c_.Resize(nn);
  diag_c_.Resize(nn);
  camdiag_.Resize(nn);
  camg_.Resize(nn);
  cslot_ = std::max(lcam_off, 1);
  cam_slab_.Resize(2 * cslot_);
  lin_scal_.Resize(2 * (size_t)std::max(nlin_, 1) * kNScal);
  S_slab_.Resize(std::max(s_off, 1));
  chunk_scal_.Resize((size_t)std::max(npu_, 1) * kNScal);
  stg.Add(pu_units_, pu_units);
  if (nk_) {
    // free intrinsics: each frame block's non-fixed observations (block NB: the fixed frames'), for k_intr_fk
    std::vector<int32_t> boff(NB_ + 2, 0), bidx;
    for (int o = 0; o < M_; ++o)
      if (!(obs_meta[o] & kMetaFixed)) {
        const int b = meta_block(obs_meta[o]);
        boff[(b >= 0 ? b : NB_) + 1] += 1;
      }
    for (int b = 0; b <= NB_; ++b) boff[b + 1] += boff[b];
    bidx.resize(std::max(boff[NB_ + 1], 1), 0);
    std::vector<int32_t> fill(boff.begin(), boff.end() - 1);
    for (int o = 0; o < M_; ++o)
      if (!(obs_meta[o] & kMetaFixed)) {
        const int b = meta_block(obs_meta[o]);
        bidx[fill[b >= 0 ? b : NB_]++] = o;
      }
    stg.Add(intr_boff_, boff);
    stg.Add(intr_bidx_, bidx);
    // slices per block list: about one observation per thread of a k_intr_fk workgroup
    int lmax = 1;
    for (int b = 0; b <= NB_; ++b) lmax = std::max(lmax, boff[b + 1] - boff[b]);
    intr_nsl_ = std::max(1, std::min(32, (lmax + 255) / 256));
  }
  if (host_timing) DevMark(s, 1);
  stg.Flush(s);
  if (host_timing) DevMark(s, 2);
  lap("flush");
  cam_wide_.Resize(2 * (size_t)std::max(NB_, 1) * kCamV);
  S_wide_.Resize(nn * nn);
  xchg_cam_.Resize(3 * ((size_t)NB_ * kCamV + kXNum + nranks()));   // summed | this rank's | candidate
  S_.Resize(nn * nn + nn + 2);   // S, then the rhs partial xc (one all-reduce covers both), then {0, 1}
  rhs_.Resize(nn);
  xchg_upd_.Resize(kUNum);
  xchg_chol_.Resize(kCNum);
  work_.Resize(nn);
  fd_r_.Resize(std::max(D_, 1));
  fd_J_.Resize(6 * (size_t)std::max(D_, 1));
  fd_D_.Resize(9 * (size_t)std::max(NB_, 1));
  fd_X_.Resize(9 * (size_t)std::max(D_, 1));
  if (nk_) {
    Jk_.Resize(14 * (size_t)std::max(M_, 1));
    KU_.Resize(nn * nk_);
    kst_.Resize(56 * (size_t)ncam_);
    Yk_.Resize(28 * (size_t)std::max(P_, 1) * ncam_);
    kpart_.Resize((size_t)(NB_ + 1) * ncam_ * 42);
  }
  stamp_on_ = getenv("SG_STAMP") && getenv("SG_STAMP")[0] == '1';
  if (stamp_on_) stamps_.Resize(kUlStamp + 16);
  lap("resize");
  ResetState(s);
  if (host_timing) DevMark(s, 3);
  lap("reset");
  WaitStream(s);
  lap("uploads");
  if (host_timing) {
    float a = 0, b = 0, c = 0;
    (void)hipEventElapsedTime(&a, dev_marks_[0], dev_marks_[1]);
    (void)hipEventElapsedTime(&b, dev_marks_[1], dev_marks_[2]);
    (void)hipEventElapsedTime(&c, dev_marks_[2], dev_marks_[3]);
    float e = 0;
    (void)hipEventElapsedTime(&e, dev_marks_[4], dev_marks_[3]);
    const double hw = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - load_t0).count();
    char buf[320];
    snprintf(buf, sizeof(buf), " [device: batch1..batch2 %.2f, scatter2 %.2f, reset %.2f; load start..reset: device "
             "%.2f, host %.2f]", a, b, c, e, hw);
    lap_log += buf;
    if (idle_valid_prev) {
      float g = 0;
      const hipError_t ge = hipEventElapsedTime(&g, ev_idle_prev_, dev_marks_[4]);
      snprintf(buf, sizeof(buf), " [last idle..load start: device %.2f (%d), host %.2f]", g, (int)ge, idle_gap_host);
      lap_log += buf;
    }
  }
  if (host_timing) {
    char buf[96];
    snprintf(buf, sizeof(buf), " (staged %.2f MB; device allocations so far %ld)", stg.staged_bytes() / 1e6,
             g_dbuf_allocs.load());
    lap_log += buf;
  }
  SaveStructure(p);
  full_loads_++;
  if (host_timing) {
    SG_HIP_CHECK(hipStreamSynchronize(stream_));
    lap("sync");
    fprintf(stderr, "[sg] Load phases (ms):%s\n", lap_log.c_str());
  }
  loaded_ = true;
  began_ = false;
  pending_decision_ = false;
}

void BaSolver::Reserve(int F, int P, int M) {
  DropGraph();
  SG_REQUIRE(F >= 0 && P >= 0 && M >= 0, SG_EINVAL, "negative reservation");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  const size_t f = std::max(F, 1), pp = std::max(P, 1), m = std::max(M, 1);
  bool moved = false;
  // per observation (device order records, the Jacobian rows, the Schur cells)
  moved |= J_.Reserve(2 * ((m + 63) & ~(size_t)63) * kJStride);
  moved |= obs_pt_.Reserve(2 * m);
  moved |= obs_frame_.Reserve(m);
  moved |= obs_fixed_.Reserve(m);
  moved |= obs_meta_.Reserve(m);
  moved |= obs_pnt_.Reserve(m);
  moved |= cells_.Reserve(4 * m);
  moved |= cell_obs_.Reserve(m);
  moved |= llist_d_.Reserve(2 * m);
  // per point
  moved |= X_.Reserve(8 * pp);
  moved |= V_.Reserve(2 * 10 * pp);
  moved |= Vinv_.Reserve(10 * pp);
  moved |= g_.Reserve(2 * 4 * pp);
  moved |= tp_.Reserve(4 * pp);
  moved |= scale_p_.Reserve(4 * pp);
  moved |= diag_p_.Reserve(4 * pp);
  moved |= pfree_.Reserve(pp);
  moved |= poff_.Reserve(pp + 1);
  moved |= pinfo_.Reserve(2 * pp);
  moved |= pmx_.Reserve(4 * pp);
  // per frame
  moved |= q_.Reserve(8 * f);
  moved |= t_.Reserve(6 * f);
  moved |= frame_cam_.Reserve(f);
  moved |= frame_block_.Reserve(f);
  moved |= rot_free_.Reserve(f);
  moved |= trans_free_.Reserve(f);
  // the pinned staging buffer and its device copy: about 51 B per observation, 93 B per point, and per frame
  // the pose slots, the FrameDistance pair table (NB^2) and the Cholesky's W tiles (2 * 8 tiles per 16 columns)
  moved |= stager_->ReserveBytes(64 * m + 128 * pp + 16384 * f + 4 * f * f + (1u << 20));
  if (moved) {   // the buffers of the loaded structure are gone: the next Load rebuilds everything
    loaded_ = false;
    began_ = false;
    skey_ = StructKey{};
  }
}

bool BaSolver::SameStructure(const sg_problem& p) const {
  const StructKey& k = skey_;
  if (p.num_cameras != k.ncam || (p.cameras_free != 0) != (k.cams_free != 0) || p.num_frames != k.F ||
      p.num_points != k.P || p.num_obs != k.M || p.num_dist != k.D)
    return false;
  auto same = [](const auto* a, const auto& v) {
    return v.empty() || std::memcmp(a, v.data(), v.size() * sizeof(v[0])) == 0;
  };
  return same(p.frame_camera, k.frame_camera) && same(p.frame_rot_free, k.rot_free) &&
         same(p.frame_trans_free, k.trans_free) && same(p.point_free, k.point_free) &&
         same(p.obs_frame, k.obs_frame) && same(p.obs_point, k.obs_point) && same(p.dist_frame, k.dist_frame) &&
         same(p.dist_prev, k.dist_prev);
}

void BaSolver::SaveStructure(const sg_problem& p) {
  StructKey& k = skey_;
  k.ncam = p.num_cameras;
  k.cams_free = p.cameras_free != 0;
  k.F = p.num_frames;
  k.P = p.num_points;
  k.M = p.num_obs;
  k.D = p.num_dist;
  k.frame_camera.assign(p.frame_camera, p.frame_camera + k.F);
  k.rot_free.assign(p.frame_rot_free, p.frame_rot_free + k.F);
  k.trans_free.assign(p.frame_trans_free, p.frame_trans_free + k.F);
  k.point_free.assign(p.point_free, p.point_free + k.P);
  k.obs_frame.assign(p.obs_frame, p.obs_frame + k.M);
  k.obs_point.assign(p.obs_point, p.obs_point + k.M);
  k.dist_frame.assign(p.dist_frame, p.dist_frame + k.D);
  k.dist_prev.assign(p.dist_prev, p.dist_prev + k.D);
}

// LM state and accumulators a fresh solve starts from (zeroed on every Load)
// Zero a few device buffers and set the tiled Cholesky's {0, 1} constants (after S and its rhs) in one launch
// (hipMemsetAsync / a pageable hipMemcpyAsync would go through the copy engine).
struct ZeroList {
  double* p[8];
  size_t n[8];   // doubles
  double* c01;   // two doubles: {0, 1}
};
__global__ __launch_bounds__(256) void k_reset_buffers(ZeroList z) {
  for (int b = 0; b < 8; ++b) {
    double* p = z.p[b];
    const size_t n = z.n[b];
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
      p[i] = 0.0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && z.c01) {
    z.c01[0] = 0.0;
    z.c01[1] = 1.0;
  }
}

void BaSolver::ResetState(hipStream_t s) {
  // LmState (slot 0 current, nothing pending: evaluate() may run before begin()), the accumulators, S; one
  // launch, no copy engine (hostmirror.h)
  ZeroList z{};
  auto put = [&](int i, void* ptr, size_t bytes) {
    z.p[i] = static_cast<double*>(ptr);
    z.n[i] = ptr ? bytes / 8 : 0;
  };
  static_assert(sizeof(LmState) % 8 == 0, "LmState is zeroed in 8-byte words");
  put(0, st_.ptr, st_.size * sizeof(LmState));
  put(1, lin_scal_.ptr, lin_scal_.size * sizeof(double));
  put(2, seg_fail_.ptr, seg_fail_.size * sizeof(*seg_fail_.ptr));
  put(3, cam_wide_.ptr, cam_wide_.size * sizeof(double));
  put(4, S_wide_.ptr, S_wide_.size * sizeof(double));
  put(5, rhs_.ptr, rhs_.size * sizeof(double));
  put(6, chunk_scal_.ptr, chunk_scal_.size * sizeof(double));
  put(7, S_.ptr, (S_.size - 2) * sizeof(double));
  z.c01 = S_.ptr + S_.size - 2;   // k_chol_tiles: padding entries of the last tile
  size_t mx = 0;
  for (int i = 0; i < 8; ++i) mx = std::max(mx, z.n[i]);
  const unsigned g = (unsigned)std::min<size_t>(512, std::max<size_t>(1, (mx + 255) / 256));
  hipLaunchKernelGGL(k_reset_buffers, dim3(g), dim3(256), 0, s, z);
  SG_HIP_CHECK(hipGetLastError());
  if (stamp_on_) stamps_.Zero(s);
}

// Same structure as the last Load: new values (poses, intrinsics, points, observed pixels, loss ranges) in
// the device order of that Load; every index list and the Cholesky envelope stay.
void BaSolver::LoadValues(const sg_problem& p) {
  range_b_ = p.range * p.range;
  fd_target_ = p.dist_target;
  fd_b2_ = p.dist_range * p.dist_range;
  stab_b_ = p.stab_range * p.stab_range;
  hipStream_t s = stream_;
  std::vector<double> k2(14 * (size_t)ncam_), q2(8 * (size_t)F_), t2(6 * (size_t)F_), X2(8 * (size_t)P_),
      obs_pt(2 * (size_t)M_);
  for (int c = 0; c < 7 * ncam_; ++c) k2[c] = k2[c + 7 * ncam_] = p.k[c];
  for (int i = 0; i < 4 * F_; ++i) q2[i] = q2[i + 4 * F_] = p.q[i];
  for (int i = 0; i < 3 * F_; ++i) t2[i] = t2[i + 3 * F_] = p.t[i];
  for (int i = 0; i < P_; ++i) {
    const int pt = point_perm_[i];
    for (int a = 0; a < 4; ++a) X2[4 * i + a] = X2[4 * (i + P_) + a] = p.X[4 * pt + a];
  }
  for (int o = 0; o < M_; ++o) {
    const int src = obs_perm_[o];
    obs_pt[2 * o] = p.obs_pt[2 * src];
    obs_pt[2 * o + 1] = p.obs_pt[2 * src + 1];
  }
  k_.Upload(k2.empty() ? std::vector<double>{0.0} : k2, s);
  q_.Upload(q2, s);
  t_.Upload(t2, s);
  X_.Upload(X2, s);
  obs_pt_.Upload(obs_pt, s);
  ResetState(s);
  SG_HIP_CHECK(hipStreamSynchronize(s));
  value_loads_++;
  loaded_ = true;
  began_ = false;
  pending_decision_ = false;
}

Dev BaSolver::MakeDev() {
  Dev d{};
  d.st = st_.ptr;
  d.k[0] = k_.ptr;
  d.k[1] = k_.ptr + 7 * (size_t)ncam_;
  d.nk = nk_;
  d.kc0 = 6 * NB_;
  d.ncam = ncam_;
  d.Jk = Jk_.ptr;
  d.KU = KU_.ptr;
  d.kst = kst_.ptr;
  d.Yk = Yk_.ptr;
  d.kpart = kpart_.ptr;
  d.intr_boff = intr_boff_.ptr;
  d.intr_bidx = intr_bidx_.ptr;
  d.stab_b = stab_b_;
  d.stab_inv_b = 1.0 / stab_b_;
  d.q[0] = q_.ptr;
  d.q[1] = q_.ptr + 4 * (size_t)F_;
  d.t[0] = t_.ptr;
  d.t[1] = t_.ptr + 3 * (size_t)F_;
  d.frame_cam = frame_cam_.ptr;
  d.frame_block = frame_block_.ptr;
  d.rot_free = rot_free_.ptr;
  d.trans_free = trans_free_.ptr;
  d.F = F_;
  d.NB = NB_;
  d.n = n_;
  d.X[0] = X_.ptr;
  d.X[1] = X_.ptr + 4 * (size_t)P_;
  d.pfree = pfree_.ptr;
  d.poff = poff_.ptr;
  d.P = P_;
  d.M = M_;
  d.obs_pt = obs_pt_.ptr;
  d.obs_frame = obs_frame_.ptr;
  d.obs_fixed = obs_fixed_.ptr;
  d.obs_meta = obs_meta_.ptr;
  d.b = range_b_;
  d.inv_b = 1.0 / range_b_;
  d.D = D_;
  d.fd_a = fd_a_.ptr;
  d.fd_b = fd_b_.ptr;
  d.fd_boff = fd_boff_.ptr;
  d.fd_bidx = fd_bidx_.ptr;
  d.fd_target = fd_target_;
  d.fd_b2 = fd_b2_;
  d.fd_inv_b2 = 1.0 / fd_b2_;
  d.fd_r = fd_r_.ptr;
  d.fd_J = fd_J_.ptr;
  d.fd_D = fd_D_.ptr;
  d.fd_X = fd_X_.ptr;
  {
    const size_t pp = std::max(P_, 1);
    for (int sl = 0; sl < 2; ++sl) {
      d.J[sl] = J_.ptr + sl * jslot_;
      d.V[sl] = V_.ptr + sl * 10 * pp;
      d.g[sl] = g_.ptr + sl * 4 * pp;
      d.cam_slab[sl] = cam_slab_.ptr + sl * cslot_;
      d.cam_wide[sl] = cam_wide_.ptr + sl * (size_t)std::max(NB_, 1) * kCamV;
      d.lin_scal[sl] = lin_scal_.ptr + sl * (size_t)std::max(nlin_, 1) * kNScal;
    }
  }
  d.spec = spec_ ? 1 : 0;
  d.scale_p = scale_p_.ptr;
  d.diag_p = diag_p_.ptr;
  d.Vinv = Vinv_.ptr;
  d.tp = tp_.ptr;
  d.scale_c = scale_c_.ptr;
  d.diag_c = diag_c_.ptr;
  d.camdiag = camdiag_.ptr;
  d.camg = camg_.ptr;
  d.cam_loff = cam_loff_.ptr;
  d.cam_lidx = cam_lidx_.ptr;
  d.s_loff = s_loff_.ptr;
  d.s_lidx = s_lidx_.ptr;
  d.r_loff = r_loff_.ptr;
  d.r_lidx = r_lidx_.ptr;
  d.S_slab = S_slab_.ptr;
  d.chunk_scal = chunk_scal_.ptr;
  d.S_wide = S_wide_.ptr;
  d.xchg_cam = xchg_cam_.ptr;
  d.xcam_loc = xchg_cam_.ptr + (size_t)NB_ * kCamV + kXNum + nranks();
  d.xchg_cand = xchg_cam_.ptr + 2 * ((size_t)NB_ * kCamV + kXNum + nranks());
  d.xtail = Spk_.ptr + npack_;
  d.rank = comm_ ? comm_->rank() : 0;
  d.nranks = nranks();
  d.S = S_.ptr;
  d.rhs = rhs_.ptr;
  d.xchg_upd = xchg_upd_.ptr;
  d.xchg_chol = xchg_chol_.ptr;
  d.xc = S_.ptr + (size_t)n_ * n_;
  d.work = work_.ptr;
  d.stamps = stamp_on_ ? stamps_.ptr : nullptr;
  d.fd_pair = fd_pair_.ptr;
  d.obs_pnt = obs_pnt_.ptr;
  d.lchunks = lchunks_d_.ptr;
  d.lrounds = lrounds_d_.ptr;
  d.llist = llist_d_.ptr;
  d.nlin = nlin_;
  d.npu = npu_;
  d.pu_units = pu_units_.ptr;
  d.segs = segs_.ptr;
  d.nseg = nseg_;
  d.sbatch = sbatch_.ptr;
  d.pinfo = reinterpret_cast<const int2*>(pinfo_.ptr);
  d.pmx = reinterpret_cast<const int4*>(pmx_.ptr);
  d.cells = reinterpret_cast<const int4*>(cells_.ptr);
  d.cell_obs = cell_obs_.ptr;
  d.wsegs = wsegs_.ptr;
  d.nwide = nwide_;
  d.stile = stile_.ptr;
  d.nstile = nstile_;
  d.seg_fail = seg_fail_.ptr;
  d.pairs = reinterpret_cast<const int2*>(pairs_.ptr);
  d.assemble = (!comm_ || comm_->rank() == 0) ? 1 : 0;
  d.dbg = getenv("SG_DBG") ? atoi(getenv("SG_DBG")) : 0;
  return d;
}

// The LM state handed over as a kernel argument (no host buffer, no copy engine: see hostmirror.h).
__global__ void k_set_state(LmState s, LmState* st) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *st = s;
}

// The current parameter slot's poses, points and intrinsics into the mapped download buffer
// [q 4F | t 3F | X 4P | k 7 ncam] (the slot is read on the device: no state round trip first).
__global__ __launch_bounds__(256) void k_download(const double* __restrict__ q, const double* __restrict__ t,
                                                  const double* __restrict__ X, const double* __restrict__ k,
                                                  const LmState* st, int F, int P, int ncam, double* __restrict__ out) {
  const int cur = st->cur;
  const size_t nq = 4 * (size_t)F, nt = 3 * (size_t)F, nx = 4 * (size_t)P, nk = 7 * (size_t)ncam;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq + nt + nx + nk;
       i += (size_t)gridDim.x * blockDim.x) {
    double v;
    if (i < nq) v = q[nq * cur + i];
    else if (i < nq + nt) v = t[nt * cur + (i - nq)];
    else if (i < nq + nt + nx) v = X[nx * cur + (i - nq - nt)];
    else v = k[nk * cur + (i - nq - nt - nx)];
    out[i] = v;
  }
}

// Wait for stream s by spinning on an event query.  hipStreamSynchronize's blocking wait returned 13-28 ms
// late in a few percent of the main.cpp replay's loads, all of whose work had been three small kernels
// (tools/e2e_replay.py, profiles/r3_v8_*); the solver's waits are short (a load, an LM batch), so the host
// spins on them, falling back to the blocking wait after SG_SPIN_MS (default 200 ms).  A sharded solver (several
// ranks, possibly rank threads or processes sharing the host's cores with the threads that run the host
// all-reduces) yields between polls and spins at most 1 ms.
void BaSolver::WaitStream(hipStream_t s) {
  static const double spin_ms = getenv("SG_SPIN_MS") ? atof(getenv("SG_SPIN_MS")) : 200.0;
  const bool shared = nranks() > 1;
  const double limit = shared ? std::min(spin_ms, 1.0) : spin_ms;
  if (!ev_wait_) SG_HIP_CHECK(hipEventCreateWithFlags(&ev_wait_, hipEventDisableTiming));
  SG_HIP_CHECK(hipEventRecord(ev_wait_, s));
  const auto t0 = std::chrono::steady_clock::now();
  while (true) {
    const hipError_t e = hipEventQuery(ev_wait_);
    if (e == hipSuccess) {
      MarkIdle(s);
      return;
    }
    if (e != hipErrorNotReady) SG_HIP_CHECK(e);
    if (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > limit) break;
    if (shared) std::this_thread::yield();
  }
  SG_HIP_CHECK(hipEventSynchronize(ev_wait_));
  MarkIdle(s);
}

// SG_HOST_TIMING: a device marker and the host clock at the moment the stream was last seen idle, so a load can
// compare the device's and the host's time from there to its first command (a late queue start shows as a
// device gap longer than the host's).
void BaSolver::MarkIdle(hipStream_t s) {
  static const bool host_timing = getenv("SG_HOST_TIMING") != nullptr;
  if (!host_timing) return;
  if (!ev_idle_) SG_HIP_CHECK(hipEventCreate(&ev_idle_));
  SG_HIP_CHECK(hipEventRecord(ev_idle_, s));
  idle_host_ = std::chrono::steady_clock::now();
  idle_valid_ = true;
}

void BaSolver::DevMark(hipStream_t s, int i) {
  if (!dev_marks_[i]) SG_HIP_CHECK(hipEventCreate(&dev_marks_[i]));
  SG_HIP_CHECK(hipEventRecord(dev_marks_[i], s));
}

void BaSolver::ReadState(LmState* h) {
  static_assert(sizeof(LmState) % 8 == 0, "LmState is copied in 8-byte words");
  mb_.Reserve(1024);
  hipLaunchKernelGGL(k_copy_u64, dim3(1), dim3(64), 0, stream_, reinterpret_cast<const unsigned long long*>(st_.ptr),
                     reinterpret_cast<unsigned long long*>(mb_.d), sizeof(LmState) / 8);
  WaitStream(stream_);
  std::memcpy(h, mb_.h, sizeof(LmState));
}

void BaSolver::Begin(const sg_solver_options& o) {
  SG_REQUIRE(loaded_, SG_EINVAL, "no problem loaded");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  const bool began_again = began_;
  if (began_) {
    // restart from the current parameter slot: move it to slot 0 (a fresh load starts in slot 0: no round trip)
    LmState h{};
    ReadState(&h);
    if (h.cur == 1) {
      SG_HIP_CHECK(hipMemcpyAsync(q_.ptr, q_.ptr + 4 * (size_t)F_, 4 * (size_t)F_ * 8, hipMemcpyDeviceToDevice, stream_));
      SG_HIP_CHECK(hipMemcpyAsync(t_.ptr, t_.ptr + 3 * (size_t)F_, 3 * (size_t)F_ * 8, hipMemcpyDeviceToDevice, stream_));
      SG_HIP_CHECK(hipMemcpyAsync(X_.ptr, X_.ptr + 4 * (size_t)P_, 4 * (size_t)P_ * 8, hipMemcpyDeviceToDevice, stream_));
      if (ncam_ > 0)
        SG_HIP_CHECK(hipMemcpyAsync(k_.ptr, k_.ptr + 7 * (size_t)ncam_, 7 * (size_t)ncam_ * 8, hipMemcpyDeviceToDevice,
                                    stream_));
    }
  }
  began_ = true;
  LmState s{};
  s.max_iter = o.max_num_iterations;
  s.max_invalid = o.max_num_consecutive_invalid_steps;
  s.disable_term = o.disable_termination;
  s.always_lin = o.always_linearize;
  s.jacobi = o.jacobi_scaling;
  s.ftol = o.function_tolerance;
  s.gtol = o.gradient_tolerance;
  s.ptol = o.parameter_tolerance;
  s.min_rel_dec = o.min_relative_decrease;
  s.max_radius = o.max_trust_region_radius;
  s.min_radius = o.min_trust_region_radius;
  s.min_diag = o.min_lm_diagonal;
  s.max_diag = o.max_lm_diagonal;
  s.cur = 0;
  s.need_lin = 1;
  s.first = 1;
  s.done = (NB_ == 0 && P_ == 0) ? 1 : 0;
  s.ok = 1;
  s.termination = s.done ? SG_FUNCTION_TOLERANCE : SG_NO_CONVERGENCE;
  s.radius = o.initial_trust_region_radius;
  s.decrease_factor = 2.0;
  hipLaunchKernelGGL(k_set_state, dim3(1), dim3(64), 0, stream_, s, st_.ptr);
  if (began_again && spec_) {
    // k_cam_reduce keeps the wide-chunk camera accumulators in speculative mode: clear both slots for the
    // restart's first k_linearize (a fresh Load has zeroed them)
    ZeroList z{};
    z.p[0] = cam_wide_.ptr;
    z.n[0] = cam_wide_.size;
    hipLaunchKernelGGL(k_reset_buffers, dim3(1), dim3(256), 0, stream_, z);
  }
  need_seq_ = true;   // the first iteration fixes the camera scale: k_schur waits for it
  pending_decision_ = false;
  for (auto& t : timers_) {
    t.total_ms = 0.0;
    t.count = 0;
  }
}

void BaSolver::TimedLaunchBegin(int id) { TimedLaunchBegin(id, stream_); }
void BaSolver::TimedLaunchEnd(int id) { TimedLaunchEnd(id, stream_); }
void BaSolver::TimedLaunchBegin(int id, hipStream_t s) {
  if (!timing_) return;
  hipEvent_t a, b;
  SG_HIP_CHECK(hipEventCreate(&a));
  SG_HIP_CHECK(hipEventCreate(&b));
  timers_[id].ev.push_back(a);
  timers_[id].ev.push_back(b);
  SG_HIP_CHECK(hipEventRecord(a, s));
}
void BaSolver::TimedLaunchEnd(int id, hipStream_t s) {
  if (!timing_) return;
  SG_HIP_CHECK(hipEventRecord(timers_[id].ev.back(), s));
}

void BaSolver::Iterate(int n) {
  SG_REQUIRE(loaded_, SG_EINVAL, "no problem loaded");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  // Graph mode (SG_GRAPH=1): one LM iteration's chain captured once per load into a hipGraph and replayed;
  // the kernels' arguments (device pointers, sizes, variant flags) are fixed between loads.  One rank, no
  // per-kernel timing, no stamps, no side stream.
  const bool graphable = graph_ok_ && !timing_ && !stamp_on_ && !(comm_ && comm_->nranks() > 1) && !pack_force_ &&
                         nk_ == 0 && !overlap_ok_ && !spec_;
  if (graphable && n > 0 && need_seq_) {   // a solve's first iteration (it linearizes) outside the graph
    EnqueueIterations(1);
    --n;
  }
  if (graphable && n > 0) {
    if (!iter_exec_) {
      hipGraph_t g = nullptr;
      SG_HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
      EnqueueIterations(1);
      SG_HIP_CHECK(hipStreamEndCapture(stream_, &g));
      const hipError_t e = hipGraphInstantiate(&iter_exec_, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      SG_HIP_CHECK(e);
    }
    for (int it = 0; it < n; ++it) SG_HIP_CHECK(hipGraphLaunch(iter_exec_, stream_));
    need_seq_ = false;
    return;
  }
  EnqueueIterations(n);
}

void BaSolver::DropGraph() {
  if (iter_exec_) (void)hipGraphExecDestroy(iter_exec_);
  iter_exec_ = nullptr;
}

void BaSolver::EnqueueIterations(int n) {
  Dev d = MakeDev();
  for (int it = 0; it < n; ++it) {
    // speculative mode: only a solve's first iteration linearizes here; later ones find the linearization of
    // the accepted point in the slot k_update_lin filled (k_linearize would exit at once: no launch)
    if (!spec_ || need_seq_) {
      TimedLaunchBegin(kKLin);
      LaunchLinearize(d);
      TimedLaunchEnd(kKLin);
    }
    // k_schur beside the camera reduction (see side_ in ba_solver.h)
    const bool first_it = need_seq_;
    const bool overlap = overlap_ok_ && !need_seq_ && nk_ == 0 && !spec_;
    need_seq_ = false;
    if (overlap) {
      SG_HIP_CHECK(hipEventRecord(ev_lin_, stream_));
      SG_HIP_CHECK(hipStreamWaitEvent(side_, ev_lin_, 0));
      TimedLaunchBegin(kKSchur, side_);
      hipLaunchKernelGGL(k_schur, dim3(std::max(nseg_, 1)), dim3(kSchurThreads), 0, side_, d, 0);
      if (nwide_) hipLaunchKernelGGL(k_schur_wide, dim3(nwide_), dim3(kSchurThreads), 0, side_, d);
      TimedLaunchEnd(kKSchur, side_);
      SG_HIP_CHECK(hipEventRecord(ev_schur_, side_));
    }
    // Landmark shards exchange twice per LM iteration after a solve's first: k_S_reduce assembles each rank's
    // own camera blocks (and, on rank 0, the FrameDistance terms) into its partial S, and the camera gradient,
    // diagonal and cost scalars ride in the same all-reduce as the band of S (k_cam_finalize modes 1 and 2);
    // the first iteration sums the camera blocks first (the Jacobi scale of the camera columns comes from
    // them), then S.  SG_XCHG_MERGE=0: the three-exchange chain every iteration; =force: the merged chain on
    // one rank too (tests the path).
    const bool multi_x = (comm_ && comm_->nranks() > 1);
    const bool merged = !first_it && nk_ == 0 && (merge_ == 2 || (multi_x && merge_ == 1));
    const int nv = NB_ * kCamV;
    // Speculative chain: the previous iteration ended with the candidate's camera reduce and the update scalars
    // (k_cam_reduce mode 1, + their all-reduce on shards); the pending decision is taken by k_cam_finalize
    // itself (one rank, or merged shards), else by k_decide, which then also makes the accepted candidate's
    // blocks current.  No pending decision (a batch's first iteration: EnqueueIterations settles it at the
    // end of every batch): the current blocks are in place.
    // One rank (no free intrinsics): the previous iteration's reduce took the decision (k_cam_reduce mode 2) and
    // this iteration's finalize pass runs inside the k_schur launch.
    const bool fin_in_schur = spec_ && !first_it && !multi_x && nk_ == 0 && !merged;
    bool decide_in_fin = false;
    if (fin_in_schur) {
      // (nothing pending: the candidate blocks of an accepted step are taken by the pass)
    } else if (spec_ && !first_it) {
      if (pending_decision_) {
        decide_in_fin = nk_ == 0 && (merged || !multi_x);
        if (!decide_in_fin) {
          TimedLaunchBegin(kKDecide);
          hipLaunchKernelGGL(k_decide, dim3(1), dim3(256), 0, stream_, d, 1);
          TimedLaunchEnd(kKDecide);
        }
        pending_decision_ = false;
      }
    } else {
      TimedLaunchBegin(kKCamReduce);
      hipLaunchKernelGGL(k_cam_reduce, dim3(NB_ + 1), dim3(kRedThreads), 0, stream_, d, 0);
      TimedLaunchEnd(kKCamReduce);
    }
    if (!merged) AllReduceSum(xchg_cam_.ptr, (size_t)nv + kXNum + nranks());
    if (nk_) {
      hipLaunchKernelGGL(k_intr_zero, dim3((std::max(n_ * nk_, (NB_ + 1) * ncam_ * 42) + 255) / 256), dim3(256), 0,
                         stream_, d);
      hipLaunchKernelGGL(k_intr_lin, dim3((std::max(M_, 1) + 255) / 256), dim3(256), 0, stream_, d);
      hipLaunchKernelGGL(k_intr_fk<0>, dim3((NB_ + 1) * intr_nsl_, ncam_), dim3(kIntrFkThreads), 0, stream_, d,
                         intr_nsl_);
      hipLaunchKernelGGL(k_intr_fin, dim3(1), dim3(kIntrFinThreads), 0, stream_, d, intr_nsl_);
    }
    if (!fin_in_schur) {
      TimedLaunchBegin(kKCamFinal);
      hipLaunchKernelGGL(k_cam_finalize, dim3(1), dim3(256), 0, stream_, d, merged ? 1 : 0, decide_in_fin ? 1 : 0);
      TimedLaunchEnd(kKCamFinal);
    }
    if (overlap) {
      SG_HIP_CHECK(hipStreamWaitEvent(stream_, ev_schur_, 0));
    } else {
      TimedLaunchBegin(kKSchur);
      hipLaunchKernelGGL(k_schur, dim3(std::max(nseg_, 1) + (fin_in_schur ? 1 : 0)), dim3(kSchurThreads), 0, stream_, d,
                         fin_in_schur ? 1 : 0);
      if (nwide_) hipLaunchKernelGGL(k_schur_wide, dim3(nwide_), dim3(kSchurThreads), 0, stream_, d);
      TimedLaunchEnd(kKSchur);
    }
    TimedLaunchBegin(kKSReduce);
    const int nwv = nstile_ + NB_;
    hipLaunchKernelGGL(k_S_reduce, dim3(std::max(nwv, 1)), dim3(256), 0, stream_, d,
                       merged ? 2 : (d.assemble ? 1 : 0));
    TimedLaunchEnd(kKSReduce);
    if (nk_) {
      hipLaunchKernelGGL(k_intr_assemble, dim3((n_ * nk_ + 255) / 256), dim3(256), 0, stream_, d);
      hipLaunchKernelGGL(k_intr_schur, dim3((std::max(P_, 1) + 127) / 128), dim3(128), 0, stream_, d);
      if (NB_ > 0)
        hipLaunchKernelGGL(k_intr_fk<1>, dim3(NB_ * intr_nsl_, ncam_), dim3(kIntrFkThreads), 0, stream_, d, intr_nsl_);
    }
    if (multi_x || pack_force_ || merged) {
      // the band of S and the rhs partial are summed over landmark shards (packed: the band only), with the
      // merged tail after them
      const int npanel = (n_ + kCholNb - 1) / kCholNb;
      const dim3 pg(npanel + 1, 4);
      TimedLaunchBegin(kKXchg);   // pack, all-reduce, unpack
      hipLaunchKernelGGL(k_S_pack, pg, dim3(256), 0, stream_, S_.ptr, n_, (const int32_t*)work_i_.ptr,
                         (const int32_t*)pack_off_.ptr, npanel, Spk_.ptr, 0);
      AllReduceSum(Spk_.ptr, npack_ + (merged ? ntail_ : 0));
      hipLaunchKernelGGL(k_S_pack, pg, dim3(256), 0, stream_, S_.ptr, n_, (const int32_t*)work_i_.ptr,
                         (const int32_t*)pack_off_.ptr, npanel, Spk_.ptr, 1);
      TimedLaunchEnd(kKXchg);
      if (merged) {
        TimedLaunchBegin(kKCamFinal);
        hipLaunchKernelGGL(k_cam_finalize, dim3(1), dim3(256), 0, stream_, d, 2, 0);
        TimedLaunchEnd(kKCamFinal);
      }
    }
    TimedLaunchBegin(kKChol);
    if (chol_tiles_)
      LaunchCholTiles(d.stamps != nullptr, CholTilesLa(), dim3(chol_nd_ > 0 ? 2 : 1), d,
                      chol_simdmap_ | (chol_cand_lds_ ? 2 : 0) | (chol_force_tmo_ ? 4 : 0));
    else if (chol_window_ && d.stamps)
      hipLaunchKernelGGL(k_cholesky_window<true>, dim3(1), dim3(kCholThreads), kCholLds, stream_, d,
                         (const int32_t*)work_i_.ptr, rdg_.ptr);
    else if (chol_window_)
      hipLaunchKernelGGL(k_cholesky_window<false>, dim3(1), dim3(kCholThreads), kCholLds, stream_, d,
                         (const int32_t*)work_i_.ptr, rdg_.ptr);
    else
      hipLaunchKernelGGL(chol_gstage_ ? k_cholesky_global<true> : k_cholesky_global<false>, dim3(1),
                         dim3(kCholThreads), (size_t)std::max(n_, 1) * 8 * (chol_gstage_ ? 1 + kCholNb : 1), stream_,
                         d, (const int32_t*)work_i_.ptr, rdg_.ptr);
    TimedLaunchEnd(kKChol);
    if (nk_) hipLaunchKernelGGL(k_intr_step, dim3(1), dim3(64), 0, stream_, d);
    TimedLaunchBegin(kKPointUpd);
    if (spec_) {
      LaunchUpdateLin(d);
    } else {
      hipLaunchKernelGGL(k_point_update, dim3(std::max(npu_, 1)), dim3(kLinThreads), 0, stream_, d);
    }
    TimedLaunchEnd(kKPointUpd);
    const bool multi = comm_ && comm_->nranks() > 1;
    // the candidate's camera blocks and linearization scalars beside the update scalars, one launch; on one rank
    // (no free intrinsics, no forced merged chain) the decision too
    const bool decide_in_reduce = !multi && nk_ == 0 && merge_ != 2;
    TimedLaunchBegin(kKUpdRed);
    if (spec_)
      hipLaunchKernelGGL(k_cam_reduce, dim3(NB_ + 2), dim3(kRedThreads), 0, stream_, d, decide_in_reduce ? 2 : 1);
    else
      hipLaunchKernelGGL(k_upd_reduce, dim3(1), dim3(kRedThreads), 0, stream_, d, multi ? 0 : 1);
    TimedLaunchEnd(kKUpdRed);
    if (multi) AllReduceSum(xchg_upd_.ptr, kUNum);
    if (spec_) {
      pending_decision_ = !decide_in_reduce;
    } else if (multi) {
      TimedLaunchBegin(kKDecide);
      hipLaunchKernelGGL(k_decide, dim3(1), dim3(256), 0, stream_, d, 0);
      TimedLaunchEnd(kKDecide);
    }
  }
  // a batch leaves no decision pending: the host's state reads and downloads see the decided step
  if (pending_decision_) {
    TimedLaunchBegin(kKDecide);
    hipLaunchKernelGGL(k_decide, dim3(1), dim3(256), 0, stream_, d, 1);
    TimedLaunchEnd(kKDecide);
    pending_decision_ = false;
  }
  SG_HIP_CHECK(hipGetLastError());
}

__global__ void k_force_linearize(LmState* st) {
  if (threadIdx.x == 0) {
    st->need_lin = 1;
    st->done = 0;
  }
}

void BaSolver::Sweep(int n) {
  SG_REQUIRE(loaded_, SG_EINVAL, "no problem loaded");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  Dev d = MakeDev();
  for (int it = 0; it < n; ++it) {
    hipLaunchKernelGGL(k_force_linearize, dim3(1), dim3(64), 0, stream_, st_.ptr);
    TimedLaunchBegin(kKLin);
    LaunchLinearize(d);
    TimedLaunchEnd(kKLin);
  }
  SG_HIP_CHECK(hipGetLastError());
}

void BaSolver::LaunchLinearize(const Dev& d) {
  const dim3 grid(std::max(nlin_, 1));
  if (lin_waves_ == 2)
    hipLaunchKernelGGL(k_linearize<2>, grid, dim3(2 * kLinThreads), 0, stream_, d);
  else
    hipLaunchKernelGGL(k_linearize<1>, grid, dim3(kLinThreads), 0, stream_, d);
}

void BaSolver::LaunchUpdateLin(const Dev& d) {
  const dim3 grid(std::max(nlin_, 1));
  if (lin_waves_ == 2) {
    if (stamp_on_)
      hipLaunchKernelGGL((k_update_lin<true, 2>), grid, dim3(2 * kLinThreads), 0, stream_, d);
    else
      hipLaunchKernelGGL((k_update_lin<false, 2>), grid, dim3(2 * kLinThreads), 0, stream_, d);
  } else {
    if (stamp_on_)
      hipLaunchKernelGGL((k_update_lin<true, 1>), grid, dim3(kLinThreads), 0, stream_, d);
    else
      hipLaunchKernelGGL((k_update_lin<false, 1>), grid, dim3(kLinThreads), 0, stream_, d);
  }
}

std::vector<unsigned long long> BaSolver::Stamps() {
  std::vector<unsigned long long> v(stamp_on_ ? stamps_.size : 64, 0);
  if (!stamp_on_) return v;
  SG_HIP_CHECK(hipMemcpyAsync(v.data(), stamps_.ptr, v.size() * 8, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
  return v;
}

void BaSolver::Sync() { SG_HIP_CHECK(hipStreamSynchronize(stream_)); }

void BaSolver::Summary(sg_solver_summary* s) {
  LmState h{};
  ReadState(&h);
  std::memset(s, 0, sizeof(*s));
  s->num_iterations = h.pushed;
  s->num_successful_steps = h.n_succ;
  s->num_unsuccessful_steps = h.n_unsucc;
  s->num_invalid_steps = h.n_invalid;
  s->termination_type = h.termination;
  s->ok = h.ok;
  s->initial_cost = h.initial_cost;
  s->final_cost = h.min_pushed_cost + h.fixed_cost;
  s->fixed_cost = h.fixed_cost;
  s->trust_region_radius = h.radius;
  s->num_lm_iterations = h.lm_iters;
  s->sync_timeouts = h.sync_timeouts;
}

void BaSolver::Download(sg_problem* p) {
  const size_t nq = 4 * (size_t)F_, nt = 3 * (size_t)F_, nx = 4 * (size_t)P_, nk = nk_ ? 7 * (size_t)ncam_ : 0;
  const size_t tot = nq + nt + nx + nk;
  mb_.Reserve(1024 + 8 * std::max<size_t>(tot, 1));
  double* out_d = reinterpret_cast<double*>(mb_.d + 1024);
  const double* out = reinterpret_cast<const double*>(mb_.h + 1024);
  const unsigned g = (unsigned)std::min<size_t>(1024, std::max<size_t>(1, (tot + 255) / 256));
  hipLaunchKernelGGL(k_download, dim3(g), dim3(256), 0, stream_, q_.ptr, t_.ptr, X_.ptr, nk ? k_.ptr : q_.ptr,
                     (const LmState*)st_.ptr, F_, P_, nk ? ncam_ : 0, out_d);
  WaitStream(stream_);
  std::copy(out, out + nq, p->q);
  std::copy(out + nq, out + nq + nt, p->t);
  const double* X = out + nq + nt;
  for (int i = 0; i < P_; ++i) {
    const int pt = point_perm_[i];
    for (int a = 0; a < 4; ++a) p->X[4 * pt + a] = X[4 * i + a];
  }
  if (nk) std::copy(out + nq + nt + nx, out + tot, p->k);
}

void BaSolver::Solve(const sg_solver_options& o, sg_problem* p, sg_solver_summary* s) {
  Begin(o);
  const int batch = 8;
  LmState h{};
  const long long cap = (long long)o.max_num_iterations * (o.max_num_consecutive_invalid_steps + 2) + 16;
  long long launched = 0;
  while (true) {
    Iterate(batch);
    launched += batch;
    ReadState(&h);
    if (h.done) break;
    SG_REQUIRE(launched < cap, SG_EDEVICE, "LM loop did not terminate on the device");
  }
  Summary(s);
  Download(p);
}

void BaSolver::Evaluate(double* residuals, double* cost, int32_t* nfail) {
  SG_REQUIRE(loaded_, SG_EINVAL, "no problem loaded");
  DBuf<double> r, c;
  DBuf<int32_t> nf;
  r.Resize(2 * (size_t)std::max(M_, 1));
  c.Resize(1);
  nf.Resize(1);
  c.Zero(stream_);
  nf.Zero(stream_);
  Dev d = MakeDev();
  if (M_ > 0)
    hipLaunchKernelGGL(k_evaluate, dim3((M_ + 255) / 256), dim3(256), 0, stream_, d, r.ptr, c.ptr, nf.ptr);
  std::vector<double> rh(2 * (size_t)M_);
  if (M_ > 0) SG_HIP_CHECK(hipMemcpyAsync(rh.data(), r.ptr, rh.size() * 8, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipMemcpyAsync(cost, c.ptr, 8, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipMemcpyAsync(nfail, nf.ptr, 4, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
  for (int o = 0; o < M_; ++o) {
    residuals[2 * obs_perm_[o]] = rh[2 * o];
    residuals[2 * obs_perm_[o] + 1] = rh[2 * o + 1];
  }
}

void BaSolver::SetTiming(bool on) {
  timing_ = on;
  for (auto& t : timers_) {
    for (auto e : t.ev) (void)hipEventDestroy(e);
    t.ev.clear();
    t.total_ms = 0.0;
    t.count = 0;
  }
}

void BaSolver::CollectTimes() {
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
  for (auto& t : timers_) {
    for (size_t i = 0; i + 1 < t.ev.size(); i += 2) {
      float ms = 0.f;
      SG_HIP_CHECK(hipEventElapsedTime(&ms, t.ev[i], t.ev[i + 1]));
      t.total_ms += ms;
      t.count += 1;
    }
    for (auto e : t.ev) (void)hipEventDestroy(e);
    t.ev.clear();
  }
}

int BaSolver::KernelTimes(char* names, int names_len, double* ms, int32_t* counts, int max) {
  CollectTimes();
  std::string all;
  int k = 0;
  for (auto& t : timers_) {
    if (k < max) {
      ms[k] = t.count ? t.total_ms / t.count : 0.0;
      counts[k] = t.count;
    }
    if (!all.empty()) all += ",";
    all += t.name;
    ++k;
  }
  if (names && names_len > 0) {
    std::strncpy(names, all.c_str(), names_len - 1);
    names[names_len - 1] = 0;
  }
  return std::min(k, max);
}

// Algorithmic bytes / flops per launch (for the roofline line in bench.py).
int BaSolver::KernelWork(double* bytes, double* flops, int max) {
  const double M = M_, P = P_, n = n_, NB = NB_;
  double npairs = 0.0;  // observation pairs of free points on free frames are not tracked here: use M*k/2
  (void)npairs;
  std::vector<double> by(kKNum, 0.0), fl(kKNum, 0.0);
  // linearize: read obs (16 B pt + 4 B frame + 1 B fixed) + point X 32 B + offsets 4 B; write J 192 B,
  // V 80 B, g 32 B per point; camera partials
  by[kKLin] = M * (16 + 4 + 1 + 192) + P * (32 + 4 + 80 + 32 + 1) + NB * kCamV * 8;
  fl[kKLin] = M * 420.0;
  by[kKSchur] = M * 192 + P * (80 + 32 + 32 + 32 + 80 + 32);
  fl[kKSchur] = 2048.0 * schur_mfma_;   // v_mfma_f64_16x16x4f64 tile updates
  by[kKPointUpd] = M * (192 + 16 + 4) + P * (32 + 32 + 80 + 32 + 32);
  if (spec_) {   // k_update_lin: the update's traffic plus the candidate's linearization (a second J record, V, g)
    by[kKPointUpd] = M * (192 + 192 + 16 + 4 + 4 + 4) + P * (32 + 32 + 80 + 32 + 32 + 80 + 32) + NB * kCamV * 8;
    fl[kKPointUpd] = M * 420.0;
  }
  by[kKChol] = n * n * 8 * 2;
  fl[kKChol] = n * n * n / 3.0;
  int k = 0;
  for (; k < std::min(max, (int)kKNum); ++k) {
    bytes[k] = by[k];
    flops[k] = fl[k];
  }
  return k;
}

void BaSolver::Info(sg_ba_info* o) const {
  std::memset(o, 0, sizeof(*o));
  o->num_frames = F_;
  o->num_points = P_;
  o->num_obs = M_;
  o->num_blocks = NB_;
  o->n = n_;
  o->band_tiles = band_tiles_;
  o->cholesky_path = chol_border_ ? 4 : chol_tiles_ ? 0 : (chol_window_ ? 1 : (chol_gstage_ ? 2 : 3));
  o->cholesky_split = chol_tiles_ ? chol_nd_ : 0;
  o->num_pairs = (int32_t)std::min<size_t>(npairs_, INT32_MAX);
  o->rank = comm_ ? comm_->rank() : 0;
  o->nranks = comm_ ? comm_->nranks() : 1;
  o->num_allreduces = nallreduce_;
  o->lin_waves = lin_waves_;
}

double BaSolver::ReprojectMap(sg_map* m) {
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  const int M = m->num_obs;
  hipStream_t s = stream_;
  mk_.Upload(std::vector<double>(m->k, m->k + 7 * m->num_cameras), s);
  mq_.Upload(std::vector<double>(m->q, m->q + 4 * m->num_frames), s);
  mt_.Upload(std::vector<double>(m->t, m->t + 3 * m->num_frames), s);
  mX_.Upload(std::vector<double>(m->X, m->X + 4 * m->num_points), s);
  mobs_pt_.Upload(std::vector<double>(m->obs_pt, m->obs_pt + 2 * M), s);
  mobs_frame_.Upload(std::vector<int32_t>(m->obs_frame, m->obs_frame + M), s);
  mobs_point_.Upload(std::vector<int32_t>(m->obs_point, m->obs_point + M), s);
  mframe_cam_.Upload(std::vector<int32_t>(m->frame_camera, m->frame_camera + m->num_frames), s);
  mobs_err_.Resize(2 * (size_t)std::max(M, 1));
  const int nb = std::max((M + 255) / 256, 1);
  mred_.Resize(2 * (size_t)nb + 2);
  mred_.Zero(s);
  if (M > 0)
    hipLaunchKernelGGL(k_reproject_map, dim3(nb), dim3(256), 0, s, mk_.ptr, mq_.ptr, mt_.ptr, mframe_cam_.ptr,
                       mX_.ptr, mobs_pt_.ptr, mobs_frame_.ptr, mobs_point_.ptr, M, mobs_err_.ptr, mred_.ptr);
  hipLaunchKernelGGL(k_reproject_reduce, dim3(1), dim3(64), 0, s, mred_.ptr, nb, mred_.ptr + 2 * nb);
  SG_HIP_CHECK(hipGetLastError());
  double out[2] = {0, 0};
  if (M > 0) SG_HIP_CHECK(hipMemcpyAsync(m->obs_error, mobs_err_.ptr, 2 * (size_t)M * 8, hipMemcpyDeviceToHost, s));
  SG_HIP_CHECK(hipMemcpyAsync(out, mred_.ptr + 2 * nb, 16, hipMemcpyDeviceToHost, s));
  SG_HIP_CHECK(hipStreamSynchronize(s));
  return out[0];
}

}  // namespace sg
