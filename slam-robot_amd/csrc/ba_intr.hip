// ba_intr.hip — the free-intrinsics columns of SolveAllFrames(..., solve_cameras = true) (slam.cpp:447-480,
// CameraStabilization slam.cpp:107-124): the 7 intrinsics of each camera as extra columns of the reduced system.
#include "ba_lm.h"

namespace sg {

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
      {
        // raw J~c (zero outside the frame's free parts): rotation pairs 1-3, translation from J~p (jc_from_pairs)
        const double2 jr[3] = {jload2(J, o, 1), jload2(J, o, 2), jload2(J, o, 3)};
        const double xw = d.X[cur][4 * (size_t)d.obs_pnt[o] + 3];
        jc_from_pairs(jr, jload2(J, o, 4), jload2(J, o, 5), jload2(J, o, 6), jload2(J, o, 7), xw, meta_tmask(m), Jc);
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
      load_scaled_J(d, J, o, b, sp, m, d.X[cur][4 * (size_t)p + 3], r, Jc, Jp);
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
      double Jr[8];   // corrected Jp (2x4; zero for a point that is not free)
      const bool pfo = (m & kMetaPfree) != 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double2 v = jload2(d.J[d.st->cur], o, 4 + i);
        Jr[2 * i] = pfo ? v.x : 0.0;
        Jr[2 * i + 1] = pfo ? v.y : 0.0;
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
// host launchers (ba_launch.h)

void LaunchIntrLinearizeK(hipStream_t s, const Dev& d, int n, int nk, int NB, int ncam, int M, int nsl) {
  hipLaunchKernelGGL(k_intr_zero, dim3((std::max(n * nk, (NB + 1) * ncam * kIntrCamV) + 255) / 256), dim3(256), 0, s,
                     d);
  hipLaunchKernelGGL(k_intr_lin, dim3((std::max(M, 1) + 255) / 256), dim3(256), 0, s, d);
  hipLaunchKernelGGL(k_intr_fk<0>, dim3((NB + 1) * nsl, ncam), dim3(kIntrFkThreads), 0, s, d, nsl);
  hipLaunchKernelGGL(k_intr_fin, dim3(1), dim3(kIntrFinThreads), 0, s, d, nsl);
}

void LaunchIntrSchurK(hipStream_t s, const Dev& d, int n, int nk, int NB, int ncam, int P, int nsl) {
  hipLaunchKernelGGL(k_intr_assemble, dim3((n * nk + 255) / 256), dim3(256), 0, s, d);
  hipLaunchKernelGGL(k_intr_schur, dim3((std::max(P, 1) + 127) / 128), dim3(128), 0, s, d);
  if (NB > 0) hipLaunchKernelGGL(k_intr_fk<1>, dim3(NB * nsl, ncam), dim3(kIntrFkThreads), 0, s, d, nsl);
}

void LaunchIntrStepK(hipStream_t s, const Dev& d) {
  hipLaunchKernelGGL(k_intr_step, dim3(1), dim3(64), 0, s, d);
}

}  // namespace sg
