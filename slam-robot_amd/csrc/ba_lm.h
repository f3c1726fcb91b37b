// ba_lm.h — the Levenberg-Marquardt bookkeeping that runs on the device (Ceres 1.8 TrustRegionMinimizer +
// LevenbergMarquardtStrategy, restated): the camera finalize pass (FrameDistance terms, cost, gradient test,
// Jacobi scale, LM diagonal) shared by k_cam_finalize and the extra workgroup of k_schur, and the step
// decision shared by k_cam_reduce mode 2, k_upd_reduce and k_decide.
#ifndef SG_BA_LM_H_
#define SG_BA_LM_H_

#include "ba_device.h"

namespace sg {

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
static __device__ void decide_step(LmState& s, const double* u, const double* c);

// The write-back of a launch whose other workgroups read LmState while one thread stores it (the concurrency
// contract in ba_kernels.h): only the fields that launch may change are stored, so the contract holds by
// construction, not by the readers' fields happening to be rewritten with the values they had.  kDecision: the
// launch takes the step decision (k_cam_reduce mode 2), which sets cur, radius, decrease_factor and reuse_diag
// for the NEXT launch (its own readers read done / spec_slot only); otherwise those stay as they are.
// spec_slot (k_update_lin's) and the options are never stored here.
template <bool kDecision>
__device__ __forceinline__ void lm_store_shared(LmState* st, const LmState& s) {
  if (kDecision) {
    st->cur = s.cur;
    st->radius = s.radius;
    st->decrease_factor = s.decrease_factor;
    st->reuse_diag = s.reuse_diag;
  }
  st->need_lin = s.need_lin;
  st->first = s.first;
  st->done = s.done;
  st->termination = s.termination;
  st->ok = s.ok;
  st->pushed = s.pushed;
  st->lm_iters = s.lm_iters;
  st->n_succ = s.n_succ;
  st->n_unsucc = s.n_unsucc;
  st->n_invalid = s.n_invalid;
  st->consecutive_invalid = s.consecutive_invalid;
  st->sync_timeouts = s.sync_timeouts;
  st->accepted = s.accepted;
  st->cost = s.cost;
  st->fixed_cost = s.fixed_cost;
  st->initial_cost = s.initial_cost;
  st->x_norm = s.x_norm;
  st->abs_gtol = s.abs_gtol;
  st->min_pushed_cost = s.min_pushed_cost;
  st->last_model = s.last_model;
  st->last_new_cost = s.last_new_cost;
  st->last_rel_decrease = s.last_rel_decrease;
  st->last_step_norm = s.last_step_norm;
}
// cam_finalize_body's write-back: k_cam_finalize runs alone (one workgroup) and may take the decision (decide 1):
// the whole struct; k_schur's finalize workgroup (decide 0 / 2, where nothing changes cur, radius, reuse_diag or
// spec_slot) runs beside the segments that read them: the contract's fields only.
__device__ __forceinline__ void fin_store(LmState* st, const LmState& s, int decide) {
  if (decide == 1)
    *st = s;
  else
    lm_store_shared<false>(st, s);
}
// LDS of the finalize pass: its own in k_cam_finalize, carved from k_schur's operand buffer when a k_schur launch
// runs it in one extra workgroup (k_schur's fin).
struct FinLds {
  double *red, *fdcost, *fdJs, *fdrs, *gsh, *dgsh, *scsh;
  int *dsh, *done_sh;
  // block_sum / block_max write red[threadIdx.x >> 6] from EVERY wave of the launch (k_schur's workgroups have
  // kSchurWaves), so red holds one slot per wave of the larger of the two workgroups
  static constexpr int kRed = kSchurWaves > 8 ? kSchurWaves : 8;
  static constexpr int kDoubles = kRed + 256 + 7 * kFinFdSh + 3 * kFinNSh + 4;
  __device__ static FinLds carve(double* p) {
    FinLds L;
    L.red = p;
    L.fdcost = p + kRed;
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
  double* red = L.red;      // FinLds::kRed slots: one per wave of the launch's workgroup
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
      if (tid == 0) fin_store(st, s0, decide);
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
      fin_store(st, s0, decide);
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
        if (decide) fin_store(st, s0, decide);   // the decision taken above (the bookkeeping follows the exchange, mode 2)
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
    if (decide && tid == 0) fin_store(st, s0, decide);
    return;
  }
  __syncthreads();
  if (tid == 0) {
    fin_count(s0);
    done_sh = s0.done;
    fin_store(st, s0, decide);
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

// The bookkeeping of k_cam_finalize mode 2 alone (merged landmark-shard chain, after the band exchange): the
// gradient max-norm of the summed camera gradient and the ranks' point maxima, Ceres's iteration push, the
// iteration count.  256 threads; red >= 4 doubles of LDS.  The damping of S's diagonal that mode 2 also does is
// applied by the unpack that runs beside it (k_S_unpack_fin).
__device__ __forceinline__ void fin_merged_bookkeeping(const Dev& d, double* red) {
  LmState* st = d.st;
  const int tid = threadIdx.x;
  const int nf = 6 * d.NB;
  const double* tg = d.xtail;
  const double* txs = d.xtail + 2 * nf;
  LmState s0;
  if (tid == 0) s0 = *st;
  const bool lin = st->need_lin;
  if (st->done) return;
  if (lin) {
    double gm = 0.0;
    for (int f = tid; f < d.F; f += 256) {
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
  if (tid == 0) {
    fin_count(s0);
    lm_store_shared<false>(st, s0);   // (k_S_unpack_fin: the unpack workgroups read LmState beside it)
  }
}

static __device__ void decide_step(LmState& s, const double* u, const double* c) {
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

}  // namespace sg

#endif  // SG_BA_LM_H_
