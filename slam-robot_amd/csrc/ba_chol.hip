// ba_chol.hip — the reduced-camera solves (the SPARSE_SCHUR + CHOLMOD step behind slam.cpp:489, restated):
// the default dissected tiled band Cholesky k_chol_tiles (MFMA trailing updates, back substitution, candidate
// poses), the bordered band of free intrinsics k_chol_border, and the window / global Cholesky for other shapes.
#include "ba_lm.h"
#include "ba_tile.h"

namespace sg {

// ------------------------------------------------------------------------------------------------
// Reduced camera system solve (the SPARSE_SCHUR + CHOLMOD step behind slam.cpp:489, restated): one
// workgroup factors the damped, banded Schur complement A = U^T U (right-looking, 16-wide panels, the
// rhs carried as an augmented column), then back-substitutes.  The band (co-visibility of the sliding
// window) fits a 128x128 fp64 LDS window that slides down the diagonal; trailing updates run as
// v_mfma_f64_16x16x4 tiles.  Bands wider than the window take the global-memory path.
constexpr int kPanelWaves = 3;   // 16 + 3 x 48 >= kCholWS columns

__device__ __forceinline__ double& Wn(double* win, int i, int j) {
  return win[(i & (kCholWS - 1)) * kCholLd + (j & (kCholWS - 1))];
}

// Wave-uniform broadcast of lane `l`'s double (v_readlane pair: no LDS round trip).
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
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
struct CandLds {
  double *q, *t, *sc, *J, *r, *tn;
  int *fb, *fl, *fa, *fbb;   // (a pair's blocks are read through fb[fa], fb[fbb]: no dependent global load)
  static size_t bytes(int F, int D, int n) {
    return (size_t)(7 * F + n + 7 * D + 3 * F) * sizeof(double) + (size_t)(2 * F + 2 * D) * sizeof(int);
  }
  __device__ void carve(double* base, int F, int D, int n) {
    q = base; t = q + 4 * F; sc = t + 3 * F; J = sc + n; r = J + 6 * D; tn = r + D;
    fb = reinterpret_cast<int*>(tn + 3 * F); fl = fb + F; fa = fl + F; fbb = fa + D;
  }
};

// Threads i0, i0 + ni, ... stage the candidate pass's operands.  With five waves or more the three lists load
// side by side: the frames on the first wave, the FrameDistance pairs on the second, the column scales on the rest.
__device__ __forceinline__ void cand_prefetch(const Dev& d, const CandLds& c, int cur, int i0, int ni) {
  int f0 = i0, fs = ni, e0 = i0, es = ni, s0 = i0, ss = ni;
  if (ni >= 5 * 64) {
    const int w = i0 >> 6, l = i0 & 63;
    f0 = w == 0 ? l : d.F;
    e0 = w == 1 ? l : d.D;
    s0 = w >= 2 ? i0 - 128 : d.n;
    fs = es = 64;
    ss = ni - 128;
  }
  for (int f = f0; f < d.F; f += fs) {
    c.fb[f] = d.frame_block[f];
    c.fl[f] = (d.rot_free[f] ? 1 : 0) | (d.trans_free[f] ? 2 : 0);
    for (int a = 0; a < 4; ++a) c.q[4 * f + a] = d.q[cur][4 * f + a];
    for (int a = 0; a < 3; ++a) c.t[3 * f + a] = d.t[cur][3 * f + a];
  }
  for (int i = s0; i < d.n; i += ss) c.sc[i] = d.scale_c[i];
  for (int e = e0; e < d.D; e += es) {
    c.fa[e] = d.fd_a[e];
    c.fbb[e] = d.fd_b[e];
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
  if (d.F <= 64 && d.D <= 64) {
    // one wave (C2: 50 frames, 49 FrameDistance pairs): a frame and a pair per lane, the sums by the wave's DPP
    // butterfly — no workgroup barrier and no LDS reduction at the end of the launch
    if (tid >= 64) return;
    double step2 = 0.0, candx2 = 0.0, model = 0.0, candcost = 0.0;
    const int f = tid;
    if (f < d.F) {
      const double* q = c.q + 4 * f;
      const double* t = c.t + 3 * f;
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
      for (int a = 0; a < 4; ++a) d.q[nxt][4 * f + a] = qq[a];
      for (int a = 0; a < 3; ++a) {
        d.t[nxt][3 * f + a] = tt[a];
        c.tn[3 * f + a] = tt[a];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's own LDS writes, in order, before its reads
    const int dd = tid;
    if (dd < d.D) {
      const int fa = c.fa[dd], fb = c.fbb[dd];
      const int ba = c.fb[fa], bb = c.fb[fb];
      const double* Jd = c.J + 6 * dd;
      double m = 0.0;
      for (int j = 0; j < 3; ++j) {
        if (ba >= 0) m += Jd[j] * c.sc[6 * ba + 3 + j] * (-y[6 * ba + 3 + j]);
        if (bb >= 0) m += Jd[3 + j] * c.sc[6 * bb + 3 + j] * (-y[6 * bb + 3 + j]);
      }
      model = -m * (c.r[dd] + 0.5 * m);
      const double* ta = c.tn + 3 * fa;
      const double* tb = c.tn + 3 * fb;
      const double e0 = ta[0] - tb[0], e1 = ta[1] - tb[1], e2 = ta[2] - tb[2];
      const double r = 0.1 * (sqrt(e0 * e0 + e1 * e1 + e2 * e2) - d.fd_target);
      double rho0, rho1;
      Cauchy(r * r, d.fd_b2, d.fd_inv_b2, &rho0, &rho1);
      candcost = 0.5 * rho0;
    }
    step2 = wave_sum_full(step2);
    candx2 = wave_sum_full(candx2);
    model = wave_sum_full(model);
    candcost = wave_sum_full(candcost);
    if (tid == 0) {
      d.xchg_chol[kCStep2] = step2;
      d.xchg_chol[kCCandX2] = candx2;
      d.xchg_chol[kCModel] = model;
      d.xchg_chol[kCCandCost] = candcost;
      d.xchg_chol[kCFail] = fail ? 1.0 : 0.0;
      d.xchg_chol[kCTimeout] = tmo ? 1.0 : 0.0;
    }
    return;
  }
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
    const int ba = c.fb[fa], bb = c.fb[fb];
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


// The owner of the next diagonal: D (acc layout) and its rhs partials -> Z, z and Z^T z of tile row K.
__device__ __forceinline__ bool tile_diag(const f64x4& D, double ypart, TileShared& sh, double* zp, int K,
                                          int lane, int li, int lk) {
#pragma unroll
  for (int q = 0; q < 4; ++q) sh.Dw[(lk + 4 * q) * kTLd + li] = (lk + 4 * q <= li) ? D[q] : 0.0;
  const double ys = sum_rows4(ypart);
  if (lk == 0) sh.Yw[li] = ys;
  double ca[kCholNb];
#ifdef SG_X_NOFACTOR   // timing-only A/B (round 6): the posts without the 16-pivot factor (results wrong)
  const bool bad = false;
#pragma unroll
  for (int r = 0; r < kCholNb; ++r) ca[r] = sh.Dw[r * kTLd + (lane & 15)];
#else
  const bool bad = tile_factor(sh.Dw, sh.Yw, sh.Id, sh.prw, ca);
#endif
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
#ifdef SG_X_ARRIVE   // diagnostic build (round 6): barrier arrivals per column offset instead of the traces
#define SG_PTRACE(K, slot) {}
#undef SG_TSTAMP
#define SG_TSTAMP(slot) {}
// per-role step stamps in registers (lane 0): late wave 0-3 (+4 arrival), owner 5-8 (+9), others 10-12 (+13)
#define SG_AST(slot)                                                             \
  if (kStamp && lane == 0) {                                                     \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();               \
    tacc[slot] += now_ - tlast;                                                  \
    tlast = now_;                                                                \
  }
#else
#define SG_AST(slot) {}
#define SG_PTRACE(K, slot)                                                                  \
  if (kStamp && lane == 0 && (K) < kTraceK)                                                \
    d.stamps[64 + ((size_t)blockIdx.x * kTraceK + (K)) * 16 + (slot)] = __builtin_amdgcn_s_memtime();
#endif

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
__device__ __forceinline__ bool la_done(const int* tend, int Kp) {   // look-ahead ran in phase Kp
  return Kp >= 0 && Kp + 2 < tend[Kp];
}

template <bool kStamp>
__device__ __forceinline__ void tile_phase(f64x4 (&acc)[kTB], double& ypart, int& J, bool& late, bool& bad,
                                           bool& tmo, TileShared& sh, const Dev& d,
                                           double* __restrict__ Wg, double* zp, const int* tend, int K, int NT,
                                           int lane, int li, int lk, const TileSrc& ts, double* zg,
                                           unsigned long long (&tacc)[16], unsigned long long& tlast) {
  if (late) {
#ifdef SG_X_NOLATE   // timing-only A/B (round 6): the late wave's W tile, reload and z' skipped (results wrong)
    J += kTB;
    late = false;
    return;
#endif
    // the previous phase's owner (column J = K): its row K-1 tile (slot 0) -> W, then column J + 8, which
    // row K + 1 touches first
    const bool hasw = J < tend[K - 1];
    f64x4 Wt = {0.0, 0.0, 0.0, 0.0};
    if (hasw) Wt = tile_w(acc[0], sh.Zs[(K - 1) & 3], li, lk);
    SG_AST(0)
    const int Jw = J;
    J += kTB;
#ifndef SG_X_NOLOAD   // timing-only A/B (round 6): no column reload (results wrong)
    tile_col_load(acc, ypart, d, J, K, li, lk, ts);
#endif
    SG_AST(1)
    if (hasw) tile_w_store(Wt, Wg, K - 1, Jw, lane);
    SG_AST(2)
    tile_zp(sh, zp, K, lane, zg);   // the diagonal this wave factored last phase
    SG_AST(3)
    late = false;
    SG_TSTAMP(13)
    return;
  }
  if (J == K + 1) SG_PTRACE(K, 8)
#ifdef SG_X_PRIO   // A/B (round 6): the owner's chain at raised issue priority over its SIMD mate
  if (J == K + 1) __builtin_amdgcn_s_setprio(3);
#endif
#ifdef SG_X_IDLE   // timing-only A/B (tools/r5_chol_ab.sh): the waves off the owner's chain do nothing
  if (J != K + 1) return;
#endif
  // (0) trailing update by row K-1 (the owner's diagonal tile, dd = 2, already took it last phase; with the
  // look-ahead its row-K tile, dd = 1, too)
#ifdef SG_X_NOTRAIL   // timing-only A/B: no trailing updates off the owner's chain
  if (K >= 1 && J < tend[K - 1] && J == K + 1) {
#else
  if (K >= 1 && J < tend[K - 1]) {
#endif
    const double* Ub = sh.Ur[(K - 1) & 1][0];
    const bool own_la = J == K + 1 && la_done(tend, K - 1);
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
  if (J == K + 1) { SG_AST(5) } else { SG_AST(10) }
  if (J == K + 1) SG_PTRACE(K, 9)
  // (1) TRSM of row K's tile
  const int te = tend[K];
  const bool act = J < te;
  const double* Zs = sh.Zs[K & 3];
  if (act) {
    const f64x4 zero = {0.0, 0.0, 0.0, 0.0};
    double za[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) za[s] = Zs[li * kTLd + 4 * s + lk];
    const f64x4 U = mfma_f64_k16(za, acc[1], zero);
    acc[1] = U;
    double* ur = sh.Ur[K & 1][J - K - 1];
#pragma unroll
    for (int q = 0; q < 4; ++q) ur[q * 64 + lane] = U[q];
    if (J == K + 1) {
      // the owner: U_{K,K+1} is the next owner's look-ahead operand (in-order LDS: data, then the flag)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&sh.uflag, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const double* zk = sh.zK[K & 3];
#pragma unroll
    for (int q = 0; q < 4; ++q) ypart = fma(-U[q], zk[lk + 4 * q], ypart);
    if (J == K + 2) {
      // next phase's owner: its diagonal tile's update by row K uses only its own U_{K,J}; apply it now,
      // off next phase's critical chain (slot 3 = row K + 2)
      double a[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) a[s] = -U[s];
      acc[3] = mfma_f64_k16(a, U, acc[3]);
      if (la_done(tend, K)) {
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
  if (J == K + 1) { SG_AST(6) } else { SG_AST(11) }
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
    SG_AST(7)
    SG_PTRACE(K, 11)
    if (K + 1 < NT) {
      bad |= tile_diag(acc[2], ypart, sh, zp, K + 1, lane, li, lk);
    }
    SG_AST(8)
#ifdef SG_X_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    SG_PTRACE(K, 12)
    late = true;
    SG_TSTAMP(11)
  } else if (act) {
    // (3) back-substitution tile
    tile_w_store(tile_w(acc[1], Zs, li, lk), Wg, K, J, lane);
    SG_AST(12)
    SG_TSTAMP(12)
  }
}

// The bottom half's step after its last factored row ND-1 (slots of phase ND): the previous owner's W tile,
// and every other wave's update of its separator column by row ND-1 ((0) of a phase, nothing else).
__device__ __forceinline__ void tile_final(f64x4 (&acc)[kTB], int J, bool& late, TileShared& sh,
                                           double* __restrict__ Wg, const int* tend, int K, int lane, int li,
                                           int lk) {
  if (late) {
    if (J < tend[K - 1]) tile_w_store(tile_w(acc[0], sh.Zs[(K - 1) & 3], li, lk), Wg, K - 1, J, lane);
    late = false;
    return;
  }
  if (J < tend[K - 1]) {
    const double* Ub = sh.Ur[(K - 1) & 1][0];
    const bool own_la = J == K + 1 && la_done(tend, K - 1);
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
// ND..ND+ns-1, rows >= ND) mapped back to S's order — reversed tile (I', J') element (a, b) is tile
// (NT-1-J', NT-1-I') element (15-b, 15-a) — in the top half's accumulator layout, and its rhs partials
// summed over the lane rows.
__device__ __forceinline__ void sep_write(const f64x4 (&acc)[kTB], double ypart, int J, int ND, int NT, int m,
                                          int ns, double* __restrict__ sepb, double* __restrict__ sepy, int li,
                                          int lk) {
  if (J < ND || J >= ND + ns) return;
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
__device__ __forceinline__ void sep_merge(f64x4 (&acc)[kTB], double& ypart, int J, int m, int ns,
                                          const double* __restrict__ sepb, const double* __restrict__ sepy,
                                          int lane, int li, int lk) {
  if (J < m || J >= m + ns) return;
  // two tiles' loads in flight per wait (unconditional loads from clamped addresses, the sums selected): written as
  // acc[u][q] += src[q * 64] the compiler waited for every load before the next (one global round trip per
  // element on the hand-off's critical path)
#pragma unroll
  for (int u0 = 0; u0 < kTB; u0 += 2) {
    f64x4 t[2];
    bool use[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = u0 + h;
      const int I = J - ((J - (u + m - 2)) & 7);   // slots of phase m - 1
      use[h] = I >= m;
      const double* src = sepb + (use[h] ? ((I - m) * 7 + (J - m)) * 256 : 0) + lane;
#pragma unroll
      for (int q = 0; q < 4; ++q) t[h][q] = src[q * 64];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (use[h])
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[u0 + h][q] += t[h][q];
  }
  if (lk == 0) ypart += sepy[(J - m) * 16 + li];
}

// The row sums of one back-substitution step, reduced and scattered: lane (li, lk) holds the partials p[q] of
// rows lk + 4q (its column li of the W tiles).  Two quad-perm exchanges leave it one of the four rows, q = 2 b0
// + b1 (b0 = li & 1, b1 = (li >> 1) & 1), summed over its quad; two row rotations (by 4 and 8 lanes) then sum the
// four quads of the lane row.  Ten DPP moves and five adds, where four full butterflies took 32 and 16.  Lanes
// li, li + 4, li + 8, li + 12 hold the same row's total, each summed in its own order: readers take it from one
// fixed lane (bs_src_lane), so every x is the same bits everywhere.
template <int kCtrl>
__device__ __forceinline__ double dpp_mv(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), kCtrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), kCtrl, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double bs_rowsum(const double (&p)[4], bool b0, bool b1) {
  const double k0 = b0 ? p[2] : p[0], k1 = b0 ? p[3] : p[1];
  const double s0 = b0 ? p[0] : p[2], s1 = b0 ? p[1] : p[3];
  const double a0 = k0 + dpp_mv<0xB1>(s0), a1 = k1 + dpp_mv<0xB1>(s1);   // quad_perm [1,0,3,2]
  const double k = b1 ? a1 : a0, sd = b1 ? a0 : a1;
  double v = k + dpp_mv<0x4E>(sd);   // quad_perm [2,3,0,1]
  v += dpp_mv<0x124>(v);             // row_ror:4
  v += dpp_mv<0x128>(v);             // row_ror:8
  return v;
}
// The lane holding row li's total after bs_rowsum (row li = lk' + 4 q', q' = li >> 2 = 2 b0' + b1').
__device__ __forceinline__ int bs_src_lane(int li) {
  const int q = li >> 2;
  return (((q >> 1) & 1) | ((q & 1) << 1)) + 16 * (li & 3);
}

// The first owner's posts when k_S_reduce has factored D_0 (flags bit 4): Z_0 (acc layout: rows lk + 4q, column
// li) into the LDS ring and z_0 = Z_0 y_0 (row sums by bs_rowsum; row r's total from one fixed lane).
__device__ __forceinline__ void tile_diag_pre(const f64x4& Z, double ypart, TileShared& sh, int li, int lk) {
  double* Zs = sh.Zs[0];
#pragma unroll
  for (int q = 0; q < 4; ++q) Zs[(lk + 4 * q) * kTLd + li] = Z[q];
  const double y = sum_rows4(ypart);   // y_0[li] in every lane
  double p[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) p[q] = Z[q] * y;
  int lb = li;
  asm volatile("" : "+v"(lb));
  const double tot = bs_rowsum(p, (lb & 1) != 0, (lb & 2) != 0);
  if (li < 4) sh.zK[0][lk + 4 * (2 * (li & 1) + ((li >> 1) & 1))] = tot;
}

// Back substitution of tile rows Khi .. Klo in one wave:  x_K = z'_K - sum_{d=1..7} W_{K,K+d} x_{K+d}, with no
// LDS round trip on the row-to-row chain.  Lane (li, lk) holds rows lk + 4q, column li of each W tile (acc
// layout) and x_{K+d}[li] in registers (xw[d-1]; zero past the last row, and W tiles outside the band are
// zero), so the d >= 2 terms are formed before x_{K+1} is known.  The 16-lane row sums are reduced and scattered
// by DPP (bs_rowsum: each lane is left one row's total), and one shuffle moves x_K[li] from its one source lane
// (bs_src_lane) to every lane.  W rows and z' are prefetched kBsBuf rows ahead
// (kBsBuf register buffers, the loop unrolled by kBsBuf).  kRev: the rows are the bottom
// half's reversed order, x_K[li] is stored at S-order index 16 (NT-1-K) + 15 - li.
#ifndef SG_BS_BUF
#define SG_BS_BUF 2
#endif
constexpr int kBsBuf = SG_BS_BUF;
template <bool kRev>
__device__ __forceinline__ void bs_chain(const double* __restrict__ Wb, const double* zsrc, double* xs, int Khi,
                                         int Klo, double (&xw)[kTB - 1], int NT, int lane, int li, int lk) {
  auto wload = [&](double (&w)[kTB - 1][4], int K) {
#ifdef SG_X_BSHOT   // timing-only A/B (round 6): every W row read from row 0 (cache-hot; results wrong)
    const double* src = Wb + (size_t)0 * (K >= 0 ? K : 0) + lane;
#else
    const double* src = Wb + (size_t)(K >= 0 ? K : 0) * kTB * 256 + lane;
#endif
#pragma unroll
    for (int dd = 1; dd < kTB; ++dd)
#pragma unroll
      for (int q = 0; q < 4; ++q) w[dd - 1][q] = src[dd * 256 + q * 64];
  };
  const int srcl = bs_src_lane(li);   // the lane holding x_K[li] after the row sums
  int lb = li;
  asm volatile("" : "+v"(lb));   // (opaque: the selects stay per-lane v_cndmask, hoisted nowhere)
  const bool b0 = (lb & 1) != 0, b1 = (lb & 2) != 0;
  const int qs = 2 * (li & 1) + ((li >> 1) & 1);   // the row lk + 4 qs this lane sums (bs_rowsum)
  // kBsBuf register buffers: row K's W tiles and z' are loaded kBsBuf rows ahead of the chain (round 6: two rows
  // ahead left the chain waiting on its L2 loads)
  auto zload = [&](double& zk, int K) { zk = zsrc[16 * (K >= 0 ? K : 0) + lk + 4 * qs]; };
  auto bs_row = [&](int K, double (&w)[kTB - 1][4], double& zk) {
    double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int dd = kTB - 1; dd >= 1; --dd)
#pragma unroll
      for (int q = 0; q < 4; ++q) p[q] = fma(w[dd - 1][q], xw[dd - 1], p[q]);
    const double xk = __shfl(zk - bs_rowsum(p, b0, b1), srcl);
    if (kRev)
      xs[16 * (NT - 1 - K) + 15 - li] = xk;
    else
      xs[16 * K + li] = xk;   // the same bits from every row of lanes
#pragma unroll
    for (int dd = kTB - 2; dd >= 1; --dd) xw[dd] = xw[dd - 1];
    xw[0] = xk;
    wload(w, K - kBsBuf);   // this buffer's next row
    zload(zk, K - kBsBuf);
  };
  double wb[kBsBuf][kTB - 1][4], zb[kBsBuf];
#pragma unroll
  for (int b = 0; b < kBsBuf; ++b) {
    wload(wb[b], Khi - b);
    zload(zb[b], Khi - b);
  }
  int K = Khi;
  for (; K >= Klo + kBsBuf - 1; K -= kBsBuf) {
#pragma unroll
    for (int b = 0; b < kBsBuf; ++b) bs_row(K - b, wb[b], zb[b]);
  }
#pragma unroll
  for (int b = 0; b < kBsBuf - 1; ++b)
    if (K - b >= Klo) bs_row(K - b, wb[b], zb[b]);
}

// The same chain on two waves (its row sums are the four full butterflies: bs_rowsum's selects push this
// variant's registers past the budget): wave `par` takes rows Khi - par, Khi - par - 2, ..., so each wave has two
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
#ifdef SG_X_BSHOT   // timing-only A/B (round 6): every W row read from row 0 (cache-hot; results wrong)
    const double* src = Wb + (size_t)0 * (K >= 0 ? K : 0) + lane;
#else
    const double* src = Wb + (size_t)(K >= 0 ? K : 0) * kTB * 256 + lane;
#endif
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

// Dissected band (nd > 0: two workgroups).  With m = NT - nd - ns, the tile rows split into the top part
// A = [0, m), the separator [m, m+ns) and the bottom part B = [m+ns, NT).  ns (flags bits 8-11, 1..7; 0 means
// 7) covers every band of A (the host picks m with max_{K<m} tend[K] = m + ns: at C2, whose rows are 6-7 tiles
// wide, a 5-row separator), so A and B never couple: eliminating A, then B, then the separator is an exact
// Cholesky of S in that order (nested dissection), and A and B are factored at the same time.
//   * blockIdx 0 (top) runs the phases of rows 0 .. m+ns-1 of S (band ends clamped to the separator); at
//     phase m-1 each wave waits for the bottom half and adds its separator contribution, then factors the
//     separator rows as usual.
//   * blockIdx 1 (bottom) runs the phases of B in reversed order (P S P: rows NT-1 .. m+7 of S, then the
//     separator as its trailing columns, started at zero), writes the separator contribution, its z' and
//     W tiles, and signals with a release counter.
//   * Back substitution (top workgroup): the separator rows, then A (wave 0) and B (wave 1, reversed W
//     tiles) side by side.
// The chain drops from NT tile rows to m + ns (C2: 18 -> 12, C5: 75 -> 42).  The wait is bounded: on a
// time-out the launch reports it (kCTimeout) and the LM decision ends the solve with SG_DEVICE_TIMEOUT
// instead of hanging or silently rejecting the step.
//   flags bit 2 (SG_CHOL_FORCE_TIMEOUT, tests only): the bottom workgroup sleeps ~2 ms before its work and
//   the top one polls at most 256 times, so the time-out path runs deterministically.
constexpr int kSepSpinMax = 1 << 22;
template <bool kStamp>
__global__ __launch_bounds__(kTileThreads) void k_chol_tiles(Dev d, const int32_t* panel_jend,
                                                             double* __restrict__ Wg, int32_t* tflag, int nd,
                                                             int flags) {
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
  const int nsf = (flags >> 8) & 15;
  const int ns = nsf > 0 && nsf < kTB ? nsf : kTB - 1;   // separator tile rows
  const int m = nd > 0 ? NT - nd - ns : NT;   // first separator tile row (S order)
  const int NTf = nd > 0 ? (bottom ? nd : m + ns) : NT;   // tile rows this workgroup factors
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
  }
  bool bad = false, tmo = false;
  const int spin_max = (flags & 4) ? 256 : kSepSpinMax;
  if (bottom && (flags & 4))
    for (int i = 0; i < 640; ++i) __builtin_amdgcn_s_sleep(127);
  // Columns J and J+1 (mod 8) on one SIMD: the owner of phase K (column K+1) then shares its SIMD with the
  // late wave of column K (one W tile, a reload) or with column K+2 (its first few tiles), not with a
  // column four ahead and its full band of trailing MFMAs.  SIMD ids from HW_ID; any other placement than
  // two waves per SIMD keeps column = wave.
  // D_0 (no updates: the wave that gets column 0 factors it first), its rhs and the LmState flag do not depend on
  // the column mapping: every wave's loads of them go out before the mapping's barrier, an LDS-only one, so they
  // stay in flight across it
  // flags bit 4: k_S_reduce has factored D_0 (the top workgroup loads Z_0 instead)
  const bool zpre_in = (flags & 16) != 0 && !bottom;
  f64x4 D0;
  bool zbad = false;
  if (zpre_in) {
#pragma unroll
    for (int q = 0; q < 4; ++q) D0[q] = d.zpre[(lk + 4 * q) * 16 + li];
    zbad = d.zpre[256] != 0.0;
  } else {
    D0 = tile_load(d.S, 0, 0, li, lk, ts);
  }
  double y0;
  {
    const int sj0 = ts.rev ? ts.np - 1 - li : li, ld = ts.ld;
    y0 = d.S[(lk == 0 && sj0 < n && 0 < ts.sep) ? ld * ld + sj0 : ld * ld + ld];
  }
  const int done = st->done;
  if (lane == 0) sh.simd[wave] = __builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);   // HW_ID.SIMD_ID
  for (int i = tid; i < 16 * kTLd; i += kTileThreads) sh.Id[i] = (i / kTLd == i % kTLd) ? 1.0 : 0.0;
  lds_barrier();
  int col = wave;
  {
    const int my = sh.simd[wave];
    int cnt[4] = {0, 0, 0, 0}, rank = 0;
#pragma unroll
    for (int w = 0; w < kTB; ++w) {
      const int sw = sh.simd[w] & 3;
      cnt[sw] += 1;
      if (w < wave && sw == my) rank += 1;
    }
#ifdef SG_X_PAIR4   // A/B (round 6): columns c and c + 4 on one SIMD
    if (cnt[0] == 2 && cnt[1] == 2 && cnt[2] == 2 && cnt[3] == 2) col = my + 4 * rank;
#else
    if (cnt[0] == 2 && cnt[1] == 2 && cnt[2] == 2 && cnt[3] == 2) col = 2 * my + rank;
#endif
  }
  {
    f64x4 acc[kTB];
    double ypart = 0.0;
    int J = col;
    bool late = false;
    // column 0's wave loads column 8 instead (D_0 is in flight) and factors D_0 while it arrives
    if (J == 0) J = kTB;
    tile_col_load(acc, ypart, d, J, 0, li, lk, ts);   // slots of phase 0
    // band ends (read first in phase 0, after the barrier below): their loads follow the column's
    for (int k = tid; k < NT; k += kTileThreads) {
      if (!bottom) {
        tend[k] = min((panel_jend[k] + 15) >> 4, NTf);
      } else {
        // reversed row k = column c = NT-1-k of S: its band reaches back to lo(c), the first row whose band
        // covers c (band ends are non-decreasing), so the reversed row ends at NT - lo(c)
        const int c = NT - 1 - k;
        // the kTB candidate rows' band ends loaded together (a loop that breaks at the first hit loaded them one
        // round trip at a time), then the first hit in row order
        int te[kTB];
#pragma unroll
        for (int h = 0; h < kTB; ++h) te[h] = panel_jend[max(0, c - kTB + h)];
        int lo = c;
#pragma unroll
        for (int h = kTB - 1; h >= 0; --h) {
          const int i = c - kTB + h;
          if (i >= 0 && ((te[h] + 15) >> 4) > c) lo = i;
        }
        tend[k] = min(NT - lo, nd + ns);
      }
    }
    if (done) return;
    if (col == 0) {
      if (zpre_in) {
        tile_diag_pre(D0, y0, sh, li, lk);
        bad |= zbad;
      } else {
        bad |= tile_diag(D0, y0, sh, zp, 0, lane, li, lk);
      }
      tile_zp(sh, zp, 0, lane, zg);   // (the wave's own LDS writes: visible to it in order)
    }
    else if (cand_lds)   // the seven waves that wait at the first barrier
      cand_prefetch(d, cl, st->cur, (col - 1) * 64 + lane, kTileThreads - 64);
    SG_TSTAMP(0)
    __syncthreads();
    SG_TSTAMP(1)
#ifdef SG_X_ARRIVE
    // per column offset d = J - K at the phase start: the cycles from this wave's phase start (barrier exit) to
    // its barrier arrival, summed / max / count (tools/arrive_trace.py)
    unsigned long long ar_sum[8] = {}, ar_max[8] = {}, ar_cnt[8] = {};
    unsigned long long t_ph = __builtin_amdgcn_s_memtime();
#endif
#pragma nounroll
    for (int K = 0; K < NTf; ++K) {
#ifdef SG_X_ARRIVE
      const int d0 = min(max(J - K, 0), 7);
      const int role = late ? 0 : (J == K + 1 ? 1 : 2);
#endif
      if (nd > 0 && !bottom && K == m - 1) {
        // relaxed polls, one acquire (an acquiring poll would invalidate the cache on every round)
        int spin = 0;
        while (__hip_atomic_load(tflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= epoch &&
               ++spin < spin_max)
          __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        tmo |= spin >= spin_max;
        sep_merge(acc, ypart, J, m, ns, sepb, sepy, lane, li, lk);
      }
      tile_phase<kStamp>(acc, ypart, J, late, bad, tmo, sh, d, Wb, zp, tend, K, NTf, lane, li, lk, ts, zg,
                         tacc, tlast);
      SG_TSTAMP(2)
      // the owner of the next diagonal (now late) is on the critical path until the barrier: it rotates after
      if (!late) tile_rotate(acc);
      SG_PTRACE(K, wave)
#ifdef SG_X_ARRIVE
      if (role == 0) { SG_AST(4) } else if (role == 1) { SG_AST(9) } else { SG_AST(13) }
      if (kStamp) {
        const unsigned long long ta = __builtin_amdgcn_s_memtime() - t_ph;
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (q == d0) {
            ar_sum[q] += ta;
            ar_max[q] = ar_max[q] > ta ? ar_max[q] : ta;
            ar_cnt[q] += 1;
          }
      }
#endif
      lds_barrier();
      if (late) tile_rotate(acc);
#ifdef SG_X_ARRIVE
      t_ph = __builtin_amdgcn_s_memtime();
      tlast = t_ph;
#endif
      SG_TSTAMP(3)
    }
#ifdef SG_X_ARRIVE
    if (kStamp && lane == 0) {
      unsigned long long* o = reinterpret_cast<unsigned long long*>(d.stamps) + kSegStamp + blockIdx.x * 256 + wave * 24;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        o[q] += ar_sum[q];
        o[8 + q] = o[8 + q] > ar_max[q] ? o[8 + q] : ar_max[q];
        o[16 + q] += ar_cnt[q];
      }
      unsigned long long* o2 = reinterpret_cast<unsigned long long*>(d.stamps) + kSegStamp + 512 + blockIdx.x * 256 +
                               wave * 16;
#pragma unroll
      for (int q = 0; q < 16; ++q) o2[q] += tacc[q];
    }
#endif
    if (bottom) {
      // row nd-1's updates of the separator columns (slots of phase nd), then the hand-off
      tile_final(acc, J, late, sh, Wb, tend, nd, lane, li, lk);
      sep_write(acc, ypart, J, nd, NT, m, ns, sepb, sepy, li, lk);
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
      if (wave == 0) bs_chain<false>(Wg, zp, xs, m + ns - 1, m, xw, NT, lane, li, lk);
      __syncthreads();
      if (wave < 2) {
#pragma unroll
        // the separator's x; past it (rows of B, solved beside this chain) zeros: A's W tiles there are zero
        for (int dd = 1; dd < kTB; ++dd) xw[dd - 1] = dd <= ns ? xs[16 * (m - 1 + dd) + li] : 0.0;
        if (m >= kBs2Rows)
          bs_chain2<false>(Wg, zp, xs, rdone, m - 1, 0, xw, NT, wave, lane, li, lk, tmo);
        else if (wave == 0)
          bs_chain<false>(Wg, zp, xs, m - 1, 0, xw, NT, lane, li, lk);
      } else if (wave < 4) {
        // x of reversed rows nd .. nd+6 (the separator, S tile rows m+6 .. m)
#pragma unroll
        for (int dd = 1; dd < kTB; ++dd) xw[dd - 1] = dd <= ns ? xs[16 * (NT - nd - dd) + 15 - li] : 0.0;
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
// Dynamic LDS (doubles): x [16 NT], z' [16 NT], row flags [NT ints], then (flags bit 0) the q_K tiles [256 NT] and
// (bit 1) the candidate pass's operands (CandLds, staged by the waves that wait for the chain).
size_t border_lds_doubles(int NT, int flags, int F, int D, int n) {
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
// host launchers (ba_launch.h)

size_t cand_lds_bytes(int F, int D, int n) { return CandLds::bytes(F, D, n); }

static const void* const kCholTilesKernels[] = {(const void*)k_chol_tiles<false>, (const void*)k_chol_tiles<true>};

void CholSetAttributes(size_t* tile_lds, size_t* gchol_lds, size_t* border_lds) {
  SG_HIP_CHECK(hipFuncSetAttribute((const void*)k_cholesky_window<false>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCholLds));
  SG_HIP_CHECK(hipFuncSetAttribute((const void*)k_cholesky_window<true>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCholLds));
  // k_chol_tiles' dynamic LDS (x, z', band ends, staged candidate operands) grows with the map: grant the most
  // the CU allows beside the kernel's static LDS
  size_t lim = 160 * 1024;
  for (const void* f : kCholTilesKernels) {
    hipFuncAttributes fa;
    SG_HIP_CHECK(hipFuncGetAttributes(&fa, f));
    lim = std::min(lim, (size_t)160 * 1024 - fa.sharedSizeBytes);
  }
  for (const void* f : kCholTilesKernels)
    SG_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lim));
  *tile_lds = lim;
  hipFuncAttributes ga;
  SG_HIP_CHECK(hipFuncGetAttributes(&ga, (const void*)k_cholesky_global<true>));
  *gchol_lds = (size_t)160 * 1024 - ga.sharedSizeBytes;
  for (const void* f : {(const void*)k_cholesky_global<true>, (const void*)k_cholesky_global<false>})
    SG_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)*gchol_lds));
  size_t blim = (size_t)160 * 1024;
  for (const void* f : {(const void*)k_chol_border<true>, (const void*)k_chol_border<false>}) {
    hipFuncAttributes ba;
    SG_HIP_CHECK(hipFuncGetAttributes(&ba, f));
    blim = std::min(blim, (size_t)160 * 1024 - ba.sharedSizeBytes);
  }
  SG_REQUIRE(border_lds_doubles(kTileMaxNT, 0, 0, 0, 0) * sizeof(double) <= blim, SG_EINVAL,
             "k_chol_border: LDS for kTileMaxNT rows");
  for (const void* f : {(const void*)k_chol_border<true>, (const void*)k_chol_border<false>})
    SG_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)blim));
  *border_lds = blim;
}

void LaunchCholTilesK(bool stamp, dim3 grid, size_t lds, hipStream_t s, const Dev& d, const int32_t* panel_jend,
                      double* Wg, int32_t* tflag, int nd, int flags) {
  Dev dd = d;
  void* args[] = {&dd, &panel_jend, &Wg, &tflag, &nd, &flags};
  SG_HIP_CHECK(hipLaunchKernel(kCholTilesKernels[stamp ? 1 : 0], grid, dim3(kTileThreads), args, lds, s));
}

void LaunchCholBorderK(int border_flags, size_t lds, hipStream_t s, const Dev& d, double* Wg) {
  hipLaunchKernelGGL((border_flags & 1) ? k_chol_border<true> : k_chol_border<false>, dim3(1), dim3(kBordThreads), lds,
                     s, d, Wg, border_flags);
}

void LaunchCholWindowK(bool stamp, hipStream_t s, const Dev& d, const int32_t* panel_jend, double* rdg) {
  if (stamp)
    hipLaunchKernelGGL(k_cholesky_window<true>, dim3(1), dim3(kCholThreads), kCholLds, s, d, panel_jend, rdg);
  else
    hipLaunchKernelGGL(k_cholesky_window<false>, dim3(1), dim3(kCholThreads), kCholLds, s, d, panel_jend, rdg);
}

void LaunchCholGlobalK(bool stage, size_t lds, hipStream_t s, const Dev& d, const int32_t* panel_jend, double* rdg) {
  hipLaunchKernelGGL(stage ? k_cholesky_global<true> : k_cholesky_global<false>, dim3(1), dim3(kCholThreads), lds, s,
                     d, panel_jend, rdg);
}

}  // namespace sg
