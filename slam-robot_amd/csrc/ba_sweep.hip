// ba_sweep.hip — the per-observation sweeps of the MI355X bundle adjustment and the LM step kernels
// (ba_launch.h lists the families): the Jacobian sweep k_linearize (project.h:11-54 + ReprojectionError,
// slam.cpp:60-84, Cauchy corrector), the speculative candidate pass k_update_lin, the two-pass chain's
// k_point_update, the deterministic camera / scalar reductions k_cam_reduce and k_upd_reduce, the step decision
// k_decide (Ceres 1.8 TrustRegionMinimizer), the residual sweep k_evaluate and ReprojectMap (slam.cpp:523-548).
#include "ba_lm.h"

namespace sg {

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

// Point accumulators in LDS (V, g of the round's points; the pass-1 terms A_p^T u): the observations of a point
// are consecutive lanes, so one LDS atomic instruction hits each of the point's addresses from ~8-10 lanes at
// once and the LDS serialises them (the point-block atomics were 22 % of k_update_lin at C2, 9 % at C5: a
// timing-only build without them, profiles/r5_s1_sweep_ab.log).  Each value has kPtCopies interleaved copies and
// lane l adds into copy l mod kPtCopies, so a point's lanes split over the copies; readers sum the copies in copy
// order (pt_sum).  Within one copy the hardware applies the lanes in lane order, so the sums stay deterministic.
// (Two copies keep the one-wave k_update_lin workgroup inside the LDS share of twelve waves per CU.)
constexpr int kPtCopies = 2;
__device__ __forceinline__ void pt_add(double* pa, int v, int lane, double x) {
  atomicAdd(pa + v * kPtCopies + (lane & (kPtCopies - 1)), x);
}
__device__ __forceinline__ double pt_sum(const double* pa, int v) {
  double s = pa[v * kPtCopies];
#pragma unroll
  for (int c = 1; c < kPtCopies; ++c) s += pa[v * kPtCopies + c];
  return s;
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
  __shared__ double pacc_w[kW][kLinPts * 14 * kPtCopies];   // point blocks of the round: V (10) | g (4), kPtCopies
                                                           // interleaved copies (pt_add)
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
  for (int i = lane; i < kLinPts * 14 * kPtCopies; i += kLinThreads) pacc[i] = 0.0;
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
      if (!ok || fx) {
        if (!ok) {
          if (fx) lsum[2][lane] += 1.0;
          else lsum[0][lane] += 1.0;
        } else if (first) {
          lsum[1][lane] += c;
        }
        jstore_zero(d.J[cur], o);
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
        // the record keeps J~p whatever the point's freedom (the translation columns come from it); the point
        // terms below use it only for a free point
        jstore(d.J[cur], o, rr, Jc, Jp);
        if (pf) {
          double* pa = pacc + (p - Rc.p0) * 14 * kPtCopies;
#pragma unroll
          for (int a = 0; a < 4; ++a) {
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
              if (cc >= a) pt_add(pa, u4(a, cc), lane, Jp[a] * Jp[cc] + Jp[4 + a] * Jp[4 + cc]);
            pt_add(pa, 10 + a, lane, Jp[a] * rr[0] + Jp[4 + a] * rr[1]);
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
        double* pa = pacc + lane * 14 * kPtCopies;
        double V[10], g[4];
#pragma unroll
        for (int i = 0; i < 10; ++i) V[i] = pt_sum(pa, i);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[i] = pt_sum(pa, 10 + i);
#pragma unroll
        for (int i = 0; i < 14 * kPtCopies; ++i) pa[i] = 0.0;
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
constexpr int kCamSlices = 32;   // (kRedThreads >= kCamSlices * kCamV)
__device__ void upd_reduce_body(const Dev& d, int fuse, int nunits);

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
    upd_reduce_body(d, mode == 2 ? 1 : 0, d.nlin);   // k_update_lin writes one unit per chunk
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
  load_scaled_J(d, d.J[cur], o, ob.b, sp, m, d.X[cur][4 * (size_t)p + 3], ob.r, Jc, ob.Jp);
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
      double* pa = pacc + (p - R.p0) * 4 * kPtCopies;
#pragma unroll
      for (int a = 0; a < 4; ++a) pt_add(pa, a, lane, ob.Jp[a] * ob.u[0] + ob.Jp[4 + a] * ob.u[1]);
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
  double* pa = pacc + 4 * kPtCopies * lane;
  double xp[4] = {0.0, 0.0, 0.0, 0.0}, Xn[4] = {X[0], X[1], X[2], X[3]};
  if (pf) {
    const double4 s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
    const double sp[4] = {s4.x, s4.y, s4.z, s4.w};
    const double4 g4 = reinterpret_cast<const double4*>(d.g[cur])[p];
    const double rhs[4] = {g4.x * sp[0] - pt_sum(pa, 0), g4.y * sp[1] - pt_sum(pa, 1), g4.z * sp[2] - pt_sum(pa, 2),
                           g4.w * sp[3] - pt_sum(pa, 3)};
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
  for (int i = 0; i < 4 * kPtCopies; ++i) pa[i] = 0.0;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
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
  __shared__ double pacc[kLinPts * 4 * kPtCopies], xps[kLinPts * 4], Xns[kLinPts * 4];
  const int lane = threadIdx.x;
  for (int i = lane; i < kLinPts * 4 * kPtCopies; i += kLinThreads) pacc[i] = 0.0;
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
// update scalars one unit per chunk (k_point_update writes one per round: the same sums in another order, so the
// two chains agree to rounding, test_ba_gpu.py::test_speculative_linearization_matches_two_pass_chain).

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
  if (!ok || fx) {
    if (!ok) lsum[fx ? 1 : 0][lane] += 1.0;   // (a fixed observation's cost counts at iteration 0 only)
    jstore_zero(d.J[nxt], o);
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
  jstore(d.J[nxt], o, rr, Jc, Jp);   // (J~p kept whatever the point's freedom; the point terms take it if free)
#ifndef SG_X_NOPATOM   // timing-only experiment build (results wrong): no point-block LDS atomics
  if (pf) {
    double* pa = pacc + lp * 14 * kPtCopies;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
#pragma unroll
      for (int cc = 0; cc < 4; ++cc)
        if (cc >= a) pt_add(pa, u4(a, cc), lane, Jp[a] * Jp[cc] + Jp[4 + a] * Jp[4 + cc]);
      pt_add(pa, 10 + a, lane, Jp[a] * rr[0] + Jp[4 + a] * rr[1]);
    }
  }
#endif
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
  double* pa = pacc + lane * 14 * kPtCopies;
  double V[10], g[4];
#pragma unroll
  for (int i = 0; i < 10; ++i) V[i] = pt_sum(pa, i);
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = pt_sum(pa, 10 + i);
#pragma unroll
  for (int i = 0; i < 14 * kPtCopies; ++i) pa[i] = 0.0;
  double2* Vd = reinterpret_cast<double2*>(d.V[nxt] + 10 * (size_t)pp);
#pragma unroll
  for (int k = 0; k < 5; ++k) Vd[k] = make_double2(V[2 * k], V[2 * k + 1]);
  reinterpret_cast<double4*>(d.g[nxt])[pp] = make_double4(g[0], g[1], g[2], g[3]);
  if (d.pfree[pp]) gmax = fmax(gmax, fmax(fmax(fabs(g[0]), fabs(g[1])), fmax(fabs(g[2]), fabs(g[3]))));
}

template <bool kStamp, int kW>
__global__ __launch_bounds__(kLinThreads * kW) SG_LIN_ATTR void k_update_lin(Dev d) {
  const LmState* st = d.st;
  const int done = st->done;
  const int cur = st->cur, nxt = cur ^ 1;
  const LinChunk ch = d.lchunks[blockIdx.x];
  // the wave's first round descriptor goes out beside LmState's, before the done test (as in k_S_reduce): at C2
  // a wave has one round, so this round trip is on the launch's critical path
  const int wv0 = threadIdx.x / kLinThreads;
  LinRound Rn{};
  if (!ch.wide && ch.r0 + wv0 < ch.r1) Rn = d.lrounds[ch.r0 + wv0];
  if (done) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) d.st->spec_slot = nxt;   // (k_cam_reduce mode 1 reads it)
  // per wave (k_linearize's split of the chunk's rounds over its waves):
  __shared__ double pacc_w[kW][kLinPts * 14 * kPtCopies];   // candidate point blocks of the round (pt_add)
  __shared__ double camacc_w[kW][kLinNbMax * kCamV];  // candidate camera blocks of the window
  __shared__ double lsum_w[kW][2][kLinThreads];       // candidate failures: free, fixed observations
  __shared__ double ua_w[kW][kLinPts * 4 * kPtCopies], xps_w[kW][kLinPts * 4], Xns_w[kW][kLinPts * 4];
  __shared__ double wscal[16];                        // wave 1's chunk scalars and update scalars
  const int lane = threadIdx.x & (kLinThreads - 1), wv = threadIdx.x / kLinThreads;
  double* pacc = pacc_w[wv];
  double* camacc = camacc_w[wv];
  double(*lsum)[kLinThreads] = lsum_w[wv];
  double* ua = ua_w[wv];     // A_p^T A_c x_c per point
  double* xps = xps_w[wv];   // x_p
  double* Xns = Xns_w[wv];   // X+
  const int ncv = ch.nb * kCamV;
  for (int i = lane; i < ncv; i += kLinThreads) camacc[i] = 0.0;
  for (int i = lane; i < kLinPts * 14 * kPtCopies; i += kLinThreads) pacc[i] = 0.0;
  for (int i = lane; i < kLinPts * 4 * kPtCopies; i += kLinThreads) ua[i] = 0.0;
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
      const LinRound R = Rn;
      if (r + kW < ch.r1) Rn = d.lrounds[r + kW];   // the next round's descriptor a round ahead
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
  }
  lds_fence_wave();
  // the update scalars of the chunk (one unit per chunk, at the chunk's index: the decision's reduction reads nlin
  // units instead of one per round, 30 k at C5, which a single workgroup took ~20 us to sum,
  // profiles/r5_s1_sweep_ab.log); the two waves' sums combined in wave order with the chunk scalars below
  double us[5] = {wave_sum_full(model), wave_sum_full(candcost), wave_sum_full(candfail), wave_sum_full(step2),
                  wave_sum_full(candx2)};
  if (kW > 1 && wv == 1 && lane == 0)
#pragma unroll
    for (int j = 0; j < 5; ++j) wscal[8 + j] = us[j];
  cost = wave_sum_full(cost);
  double fail = wave_sum_full(lsum[0][lane]);
  double ffail = wave_sum_full(lsum[1][lane]);
  gmax = wave_max_full(gmax);
  // the same combine as k_linearize's (its fixed and |X|^2 sums are zero here)
  double fixed = 0.0, xn2 = 0.0;
  lin_combine_waves<kW>(d.cam_slab[nxt] + ch.cam_off, camacc_w, ncv, wscal, wv, lane, cost, fail, fixed, ffail,
                        xn2, gmax);
  if (wv == 0 && lane == 0) {
    {
      double* su = d.chunk_scal + blockIdx.x;   // structure of arrays: slot j at [j * npu + chunk]
      const size_t nu = d.npu;
      if (kW > 1)
#pragma unroll
        for (int j = 0; j < 5; ++j) us[j] += wscal[8 + j];
      su[kModel * nu] = us[0];
      su[kCandCost * nu] = us[1];
      su[kCandFail * nu] = us[2];
      su[kStep2 * nu] = us[3];
      su[kCandX2 * nu] = us[4];
    }
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


// fuse: single rank, no all-reduce in between: thread 0 also runs k_decide's step (one launch less).
__global__ __launch_bounds__(kRedThreads) void k_upd_reduce(Dev d, int fuse) { upd_reduce_body(d, fuse, d.npu); }

// nunits: the work units whose update scalars are summed (k_point_update's rounds, or k_update_lin's chunks)
__device__ void upd_reduce_body(const Dev& d, int fuse, int nunits) {
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
  for (int c0 = tid; c0 < nunits; c0 += kUpdU * kRedThreads) {
    double t[kUpdU][5];
#pragma unroll
    for (int u = 0; u < kUpdU; ++u) {
      const int c = c0 + u * kRedThreads;
      const double* sc = d.chunk_scal + (c < nunits ? c : 0);   // coalesced: slot j at [j * npu + unit]
      const size_t ns = d.npu;
      t[u][0] = sc[kModel * ns];
      t[u][1] = sc[kCandCost * ns];
      t[u][2] = sc[kCandFail * ns];
      t[u][3] = sc[kStep2 * ns];
      t[u][4] = sc[kCandX2 * ns];
    }
#pragma unroll
    for (int u = 0; u < kUpdU; ++u)
      if (c0 + u * kRedThreads < nunits) {
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
      lm_store_shared<true>(d.st, s);   // k_cam_reduce mode 2: workgroups 0..NB read done / spec_slot beside it
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


// ------------------------------------------------------------------------------------------------
// host launchers (ba_launch.h)

void LaunchLinearizeK(int waves, int grid, hipStream_t s, const Dev& d) {
  if (waves == 2)
    hipLaunchKernelGGL(k_linearize<2>, dim3(grid), dim3(2 * kLinThreads), 0, s, d);
  else
    hipLaunchKernelGGL(k_linearize<1>, dim3(grid), dim3(kLinThreads), 0, s, d);
}

void LaunchUpdateLinK(bool stamp, int waves, int grid, hipStream_t s, const Dev& d) {
  if (waves == 2) {
    if (stamp)
      hipLaunchKernelGGL((k_update_lin<true, 2>), dim3(grid), dim3(2 * kLinThreads), 0, s, d);
    else
      hipLaunchKernelGGL((k_update_lin<false, 2>), dim3(grid), dim3(2 * kLinThreads), 0, s, d);
  } else {
    if (stamp)
      hipLaunchKernelGGL((k_update_lin<true, 1>), dim3(grid), dim3(kLinThreads), 0, s, d);
    else
      hipLaunchKernelGGL((k_update_lin<false, 1>), dim3(grid), dim3(kLinThreads), 0, s, d);
  }
}

void LaunchPointUpdateK(int grid, hipStream_t s, const Dev& d) {
  hipLaunchKernelGGL(k_point_update, dim3(grid), dim3(kLinThreads), 0, s, d);
}

void LaunchCamReduceK(int grid, hipStream_t s, const Dev& d, int mode) {
  hipLaunchKernelGGL(k_cam_reduce, dim3(grid), dim3(kRedThreads), 0, s, d, mode);
}

void LaunchUpdReduceK(hipStream_t s, const Dev& d, int fuse) {
  hipLaunchKernelGGL(k_upd_reduce, dim3(1), dim3(kRedThreads), 0, s, d, fuse);
}

void LaunchDecideK(hipStream_t s, const Dev& d, int take) {
  hipLaunchKernelGGL(k_decide, dim3(1), dim3(256), 0, s, d, take);
}

void LaunchEvaluateK(int M, hipStream_t s, const Dev& d, double* resid, double* cost, int32_t* nfail) {
  hipLaunchKernelGGL(k_evaluate, dim3((M + 255) / 256), dim3(256), 0, s, d, resid, cost, nfail);
}

void LaunchReprojectMapK(int M, int nb, hipStream_t s, const double* k, const double* q, const double* t,
                         const int32_t* frame_cam, const double* X, const double* obs_pt, const int32_t* obs_frame,
                         const int32_t* obs_point, double* err, double* partial) {
  hipLaunchKernelGGL(k_reproject_map, dim3(nb), dim3(256), 0, s, k, q, t, frame_cam, X, obs_pt, obs_frame,
                     obs_point, M, err, partial);   // (M = 0: one block writes a zero partial)
  hipLaunchKernelGGL(k_reproject_reduce, dim3(1), dim3(64), 0, s, partial, nb, partial + 2 * nb);
}

}  // namespace sg
