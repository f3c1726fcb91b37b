// ba_device.h — device-side helpers shared by the bundle-adjustment kernel families (ba_sweep.hip,
// ba_schur.hip, ba_chol.hip, ba_intr.hip): DPP / permlane wave sums, deterministic block reductions, the packed
// upper-triangle index maps, the Jacobian record layout and the 4x4 point-block inverse.
#ifndef SG_BA_DEVICE_H_
#define SG_BA_DEVICE_H_

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>

#include "ba_kernels.h"
#include "ba_launch.h"
#include "common.h"
#include "project_math.h"
#include "schur_tiles.h"

namespace sg {

#ifndef SG_LIN_ATTR
#define SG_LIN_ATTR
#endif

// ------------------------------------------------------------------------------------------------
// small device helpers


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

// Observation records J in blocks of 64 observations, element pairs interleaved: pair e2 (0..kJPairs-1) of
// observation o at double2 index ((o >> 6) * kJPairs + e2) * 64 + (o & 63).  A wave's lanes reading (or writing)
// one element pair of 64 consecutive observations touch one contiguous KiB instead of a 16-byte piece of 64
// different records.  Pairs: 0 r~ | 1-3 the rotation columns of J~c (rows 0, 1: J~c[0..2], J~c[6..8]; zero unless
// the frame's rotation is free) | 4-7 J~p (2 x 4), stored for every observation whatever the point's freedom.
// The translation columns are not stored: project.h's d(uv)/dt = -X.w d(uv)/d(X.xyz), so J~t = -X.w J~p[:, 0:3]
// (LinearizeObservation forms them that way, so every reader gets the same bits) — 128 bytes per observation
// instead of 192 (round 6).
__device__ __forceinline__ size_t jidx2(int o, int e2) { return ((size_t)(o >> 6) * kJPairs + e2) * 64 + (o & 63); }
__device__ __forceinline__ double2 jload2(const double* J, int o, int e2) {
  return reinterpret_cast<const double2*>(J)[jidx2(o, e2)];
}
// Write one observation's record (rr, Jc rotation columns, Jp) — the translation columns are implied.
__device__ __forceinline__ void jstore(double* J, int o, const double* rr, const double* Jc, const double* Jp) {
  double2* Jo = reinterpret_cast<double2*>(J) + jidx2(o, 0);   // pair e2 at Jo[64 e2]
  Jo[0] = make_double2(rr[0], rr[1]);
  Jo[64 * 1] = make_double2(Jc[0], Jc[1]);
  Jo[64 * 2] = make_double2(Jc[2], Jc[6]);
  Jo[64 * 3] = make_double2(Jc[7], Jc[8]);
#pragma unroll
  for (int i = 0; i < 4; ++i) Jo[64 * (4 + i)] = make_double2(Jp[2 * i], Jp[2 * i + 1]);
}
__device__ __forceinline__ void jstore_zero(double* J, int o) {
  double2* Jo = reinterpret_cast<double2*>(J) + jidx2(o, 0);
#pragma unroll
  for (int i = 0; i < kJPairs; ++i) Jo[64 * i] = make_double2(0.0, 0.0);
}
// The unscaled J~c (2 x 6, row-major) of a record from its pairs 1-3 (rotation) and 4-5 (J~p[:, 0:3]), the
// translation columns -X.w J~p[:, c] when the frame's translation is free (tmask), else zero.
__device__ __forceinline__ void jc_from_pairs(const double2 (&jr)[3], const double2& p4, const double2& p5,
                                              const double2& p6, const double2& p7, double xw, bool tmask,
                                              double* Jc) {
  Jc[0] = jr[0].x; Jc[1] = jr[0].y; Jc[2] = jr[1].x;
  Jc[6] = jr[1].y; Jc[7] = jr[2].x; Jc[8] = jr[2].y;
  const double nx = -xw;
  Jc[3] = tmask ? nx * p4.x : 0.0;
  Jc[4] = tmask ? nx * p4.y : 0.0;
  Jc[5] = tmask ? nx * p5.x : 0.0;
  Jc[9] = tmask ? nx * p6.x : 0.0;
  Jc[10] = tmask ? nx * p6.y : 0.0;
  Jc[11] = tmask ? nx * p7.x : 0.0;
}
__device__ __forceinline__ bool meta_tmask(int m) { return (m & kMetaTrans) != 0 && meta_block(m) >= 0; }

// Load the corrected Jacobian of observation o (meta m, its point's X.w) and apply Jacobi scaling; J~p is zero
// for a point that is not free, J~c for an observation of a frame without a free block.
__device__ __forceinline__ void load_scaled_J(const Dev& d, const double* J, int o, int b, const double* sp,
                                              int m, double xw, double* r, double* Jc, double* Jp) {
  double2 v[kJPairs];
#pragma unroll
  for (int i = 0; i < kJPairs; ++i) v[i] = jload2(J, o, i);
  r[0] = v[0].x;
  r[1] = v[0].y;
  if (b >= 0) {
    const double2 jr[3] = {v[1], v[2], v[3]};
    double Jraw[12];
    jc_from_pairs(jr, v[4], v[5], v[6], v[7], xw, meta_tmask(m), Jraw);
    const double* sc = d.scale_c + 6 * b;
#pragma unroll
    for (int i = 0; i < 12; ++i) Jc[i] = Jraw[i] * sc[i % 6];
  } else {
#pragma unroll
    for (int i = 0; i < 12; ++i) Jc[i] = 0.0;
  }
  const bool pf = (m & kMetaPfree) != 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    Jp[2 * i] = pf ? v[4 + i].x * sp[(2 * i) % 4] : 0.0;
    Jp[2 * i + 1] = pf ? v[4 + i].y * sp[(2 * i + 1) % 4] : 0.0;
  }
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


}  // namespace sg

#endif  // SG_BA_DEVICE_H_
