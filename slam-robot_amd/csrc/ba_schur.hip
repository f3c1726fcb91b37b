// ba_schur.hip — point elimination and reduced-camera-system assembly (the SchurEliminator of Ceres 1.8's
// SPARSE_SCHUR behind slam.cpp:489, restated on the matrix cores): k_schur (whitened point Jacobians, one
// v_mfma_f64_16x16x4f64 per point and tile of S), k_schur_wide, the fixed-order reduce k_S_reduce, the landmark
// shards' band packing k_S_pack, and the camera finalize pass k_cam_finalize (FrameDistance, slam.cpp:86-105).
#include "ba_lm.h"
#include "ba_tile.h"

namespace sg {

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

// J~c of observation o (block b >= 0, point X.w xw) with Jacobi scaling: its rotation pairs and the translation
// columns -X.w J~p[:, 0:3] (ba_device.h jc_from_pairs; load_scaled_J's arithmetic)
__device__ __forceinline__ void load_Jc_scaled(const Dev& d, const double* J, int o, int b, double xw, double* Jc) {
  const double* sc = d.scale_c + 6 * b;
  const double2 jr[3] = {jload2(J, o, 1), jload2(J, o, 2), jload2(J, o, 3)};
  double Jraw[12];
  jc_from_pairs(jr, jload2(J, o, 4), jload2(J, o, 5), jload2(J, o, 6), jload2(J, o, 7), xw,
                meta_tmask(d.obs_meta[o]), Jraw);
#pragma unroll
  for (int i = 0; i < 12; ++i) Jc[i] = Jraw[i] * sc[i % 6];
}
// J~p of observation o of a free point, scaled
__device__ __forceinline__ void load_Jp_scaled(const double* J, int o, const double4& s4, double* Jp) {
  const double sp[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double2 v = jload2(J, o, 4 + i);   // (pairs 0-3: r, rotation)
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
  double w[3][kSchurBatchPts * 5];           // w = L^-1 g~ and a zero per point (schur_fetch)
  int4 pinf[3][kSchurBatchPts];              // first block, span, operand offset | (jhi + 1) << 20, last window
                                             // tile jhi
  int2 pob[3][kSchurBatchPts];               // observation of its first block (-1: cell records), first cell
  uint8_t cmap[3][kSchurBatchCells];         // batch-local cell -> point
  double red[kSchurThreads / 64];
};

// The point wave's inputs for one point (thread t of batch B), loaded one batch ahead of their use so that their
// memory latency overlaps the previous batch's arithmetic; LmState's fields the pass reads are fixed for the
// launch (ba_kernels.h's contract) and read once.
struct PointPrm {
  int cur, reuse;
  double radius, min_diag, max_diag;
};
struct PointIn {
  int2 pi;
  int4 pm;
  int free;
  double V[10];
  double4 s4, g4, d4;
};
__device__ __forceinline__ void point_load(const Dev& d, const PointPrm& pr, const SchurBatch& B, int t, PointIn& in) {
  in.free = 0;
  if (t >= B.p1 - B.p0) return;
  const int p = B.p0 + t;
  in.pi = d.pinfo[p];
  in.pm = d.pmx[p];
  in.free = d.pfree[p];
  const double* Vp = d.V[pr.cur] + 10 * (size_t)p;
#pragma unroll
  for (int i = 0; i < 10; ++i) in.V[i] = Vp[i];
  in.s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
  in.g4 = reinterpret_cast<const double4*>(d.g[pr.cur])[p];
  if (pr.reuse) in.d4 = reinterpret_cast<const double4*>(d.diag_p)[p];
}
// The first batch's loads from the segment descriptor alone (the batch starts at the segment's first point), so
// they do not wait for the batch descriptor: lanes past the batch but inside the segment load real points that
// point_finish then skips (it tests the batch's count first).
__device__ __forceinline__ void point_load_first(const Dev& d, const PointPrm& pr, int p0, int pend, int t,
                                                 PointIn& in) {
  in.free = 0;
  const int p = p0 + t;
  if (p >= pend) return;
  in.pi = d.pinfo[p];
  in.pm = d.pmx[p];
  in.free = d.pfree[p];
  const double* Vp = d.V[pr.cur] + 10 * (size_t)p;
#pragma unroll
  for (int i = 0; i < 10; ++i) in.V[i] = Vp[i];
  in.s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
  in.g4 = reinterpret_cast<const double4*>(d.g[pr.cur])[p];
  if (pr.reuse) in.d4 = reinterpret_cast<const double4*>(d.diag_p)[p];
}
// point_block's arithmetic on preloaded inputs, then the point's table entries and cell map
__device__ __forceinline__ double point_finish(const Dev& d, const PointPrm& pr, const SchurBatch& B, int t,
                                               const PointIn& in, double* Lsh, double* wsh, int4* pinf, int2* pob,
                                               uint8_t* cmap) {
  if (t >= B.p1 - B.p0) return 0.0;
  const int p = B.p0 + t;
  int span = in.pi.y & 0xff, jhi = in.pm.y;
  double fail = 0.0;
  if (in.free) {
    const double sp[4] = {in.s4.x, in.s4.y, in.s4.z, in.s4.w};
    const double gs[4] = {in.g4.x * sp[0], in.g4.y * sp[1], in.g4.z * sp[2], in.g4.w * sp[3]};
    double dp[4];
    if (!pr.reuse) {
#pragma unroll
      for (int a = 0; a < 4; ++a) dp[a] = fmin(fmax(sp[a] * sp[a] * in.V[u4(a, a)], pr.min_diag), pr.max_diag);
      reinterpret_cast<double4*>(d.diag_p)[p] = make_double4(dp[0], dp[1], dp[2], dp[3]);
    } else {
      dp[0] = in.d4.x; dp[1] = in.d4.y; dp[2] = in.d4.z; dp[3] = in.d4.w;
    }
    double Vt[10], Vi[10], Li[10];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c >= a) Vt[u4(a, c)] = sp[a] * in.V[u4(a, c)] * sp[c] + (a == c ? dp[a] / pr.radius : 0.0);
    if (!inv4_spd(Vt, Vi, Li)) {
      fail = 1.0;
#pragma unroll
      for (int i = 0; i < 10; ++i) Vi[i] = Li[i] = NAN;
    }
    double tp[4], w[4];
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
#pragma unroll
    for (int i = 0; i < 10; ++i) Lsh[10 * t + i] = Li[i];
#pragma unroll
    for (int a = 0; a < 4; ++a) wsh[5 * t + a] = w[a];
    wsh[5 * t + 4] = 0.0;
  } else {
    span = 0;
    jhi = -1;
  }
  pinf[t] = make_int4(in.pi.y >> 8, span, in.pm.x | ((jhi + 1) << 20), jhi);
  pob[t] = make_int2(in.pm.z, in.pm.w);
  for (int k = 0; k < span; ++k) cmap[in.pm.w + k] = (uint8_t)t;
  return fail;
}

// Cell waves: thread per cell (point p, block b) of batch B.  E_{p,b} = sum_o G_o J~c,o with
// G_o = L^-1 J~p,o^T (4 x 2), written straight into the point's operand tiles: window column c = 6 b + a - c0w
// goes to tile c >> 4, lane (c & 15) + 16 k.  A point observed once in every block of its span (obs sorted by
// block at load) finds its observation at a fixed offset; others read the cell records.  The cells of a point
// also zero the columns of its tiles 0 .. jhi outside its span (its margins), dealt round-robin over them.
// Each thread takes two cells per round and issues the loads of both (the common single-observation cells:
// J pairs and scales) before either's arithmetic, so two cells' memory latencies overlap (the same
// arithmetic in the same order as one cell at a time: the same bits).
struct CellOps {
  double2 jp[4], jr[3];
  double4 s4;
  double sc[6];
  double xw;   // the point's X.w (the translation columns are -X.w J~p[:, 0:3])
  int tm;      // the frame's translation is free
};
__device__ __forceinline__ void cell_load(const Dev& d, const double* J, const double* X, int o, int b, int p,
                                          CellOps& c) {
#pragma unroll
  for (int i = 0; i < 4; ++i) c.jp[i] = jload2(J, o, 4 + i);   // (pairs 0-3: r, rotation)
#pragma unroll
  for (int i = 0; i < 3; ++i) c.jr[i] = jload2(J, o, 1 + i);   // (pair 0: r)
  c.s4 = reinterpret_cast<const double4*>(d.scale_p)[p];
#pragma unroll
  for (int i = 0; i < 6; ++i) c.sc[i] = d.scale_c[6 * b + i];
  c.xw = X[4 * (size_t)p + 3];
  c.tm = meta_tmask(d.obs_meta[o]) ? 1 : 0;
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
  {
    double Jraw[12];
    jc_from_pairs(c.jr, c.jp[0], c.jp[1], c.jp[2], c.jp[3], c.xw, c.tm != 0, Jraw);
#pragma unroll
    for (int i = 0; i < 12; ++i) Jc[i] = Jraw[i] * c.sc[i % 6];
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
__device__ __forceinline__ void schur_cells(const Dev& d, const double* J, const double* X, const SchurBatch& B,
                                            int tid, int c0w,
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
          cell_load(d, J, X, oc[h], bc[h], B.p0 + t, ops[h]);
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
      double* xp = Xb + (pi.z & 0xfffff);
      const int col0 = 6 * b - c0w;
      auto at = [&](int col, int k) -> double& { return xp[64 * (col >> 4) + 16 * k + (col & 15)]; };
      {
        // the point's margins — the columns of its tiles 0 .. jhi outside its span, which the consumer reads —
        // zeroed by all of its span cells, margin column m by cell m mod span (one cell per margin used to take
        // them all: 40 % of the cell waves' time at C5, profiles/r5_s1_schur_ab.log)
        const int q = b - pi.x, lo = 6 * pi.x - c0w, hi = lo + 6 * pi.y, nl = lo, nm = lo + 16 * (pi.w + 1) - hi;
        for (int m = q; m < nm; m += pi.y) {
          const int col = m < nl ? m : hi + (m - nl);
#pragma unroll
          for (int k = 0; k < 4; ++k) at(col, k) = 0.0;
        }
      }
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
        cell_load(d, J, X, o, b, B.p0 + t, c);
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
  static_assert(FinLds::kDoubles <= sizeof(sh.X) / sizeof(double), "the finalize pass's LDS fits the operand buffer");
  if (fin && blockIdx.x == 0) {
    // fin 1 (one rank): the full pass, taking an accepted step's candidate blocks (decide 2); fin 2 (merged
    // landmark shards): this rank's camera gradient / diagonal and FrameDistance terms into the exchange tail
    // (mode 1; the decision was taken by k_decide before this launch)
    cam_finalize_body(d, fin == 2 ? 1 : 0, fin == 2 ? 0 : 2, FinLds::carve(&sh.X[0][0]));
    return;
  }
  const int seg = (int)blockIdx.x - (fin ? 1 : 0);
  if (seg >= d.nseg) return;
  unsigned long long last_ = __builtin_amdgcn_s_memtime();
  // per-segment stamps (a variant build with -DSG_SEG_STAMPS, run with SG_STAMP=1; segments < kSegStampMax,
  // tools/schur_seg_stamps.py): the workgroup's span and each wave group's busy cycles (work between barriers)
#ifdef SG_SEG_STAMPS
  const bool sstamp = d.stamps != nullptr && seg < kSegStampMax;
  const unsigned long long t_wg = last_;
  unsigned long long busy = 0, tb = 0;
#define SG_BUSY_BEGIN if (sstamp) tb = __builtin_amdgcn_s_memtime();
#define SG_BUSY_END if (sstamp) busy += __builtin_amdgcn_s_memtime() - tb;
#else
#define SG_BUSY_BEGIN
#define SG_BUSY_END
#endif
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
      SG_BUSY_BEGIN
      if (s < nbt)
        schur_cells(d, d.J[st->cur], d.X[st->cur], d.sbatch[sg.bt0 + s], tid, c0w, sh.L[s % 3], sh.pinf[s % 3], sh.pob[s % 3], sh.cmap[s % 3],
                    sh.X[s & 1]);
      SG_BUSY_END
      SG_SSTAMP(34)
      __syncthreads();
      SG_SSTAMP(36)
    }
  } else if (wave == kSchurCellWaves) {
    // the point wave: batch k's point blocks in step k - 1, its inputs loaded in step k - 2
    SG_BUSY_BEGIN
    const PointPrm pr{st->cur, st->reuse_diag, st->radius, st->min_diag, st->max_diag};
    PointIn pin, pnx;
    SchurBatch Bk{}, Bn{};
    if (nbt > 0) {
      Bk = d.sbatch[sg.bt0];
      point_load_first(d, pr, sg.p0, sg.p1, lane, pin);
    }
    if (nbt > 1) {
      Bn = d.sbatch[sg.bt0 + 1];
      point_load(d, pr, Bn, lane, pnx);
    }
    if (nbt > 0) linfail += point_finish(d, pr, Bk, lane, pin, sh.L[0], sh.w[0], sh.pinf[0], sh.pob[0], sh.cmap[0]);
    SG_BUSY_END
    __syncthreads();
    for (int s = 0; s <= nbt; ++s) {
      SG_BUSY_BEGIN
      if (s + 1 < nbt) {
        const int q = (s + 1) % 3;
        Bk = Bn;
        pin = pnx;
        if (s + 2 < nbt) {
          Bn = d.sbatch[sg.bt0 + s + 2];
          point_load(d, pr, Bn, lane, pnx);
        }
        linfail += point_finish(d, pr, Bk, lane, pin, sh.L[q], sh.w[q], sh.pinf[q], sh.pob[q], sh.cmap[q]);
      }
      SG_BUSY_END

      SG_SSTAMP(35)
      __syncthreads();
      SG_SSTAMP(37)
    }
  } else {
    // MFMA waves: wave cw owns the augmented window slots u = cw + kSchurCWaves s
    const int cw = wave - kSchurCellWaves - 1;
    f64x4 acc[kSchurTPW];      // window-tile slots
    double accr[kSchurTPW];    // rhs slots (schur_chain.h)
#pragma unroll
    for (int s = 0; s < kSchurTPW; ++s) {
      acc[s] = f64x4{0.0, 0.0, 0.0, 0.0};
      accr[s] = 0.0;
    }
    SG_SSTAMP(40)
    __syncthreads();
    SG_SSTAMP(41)
    for (int s = 0; s <= nbt; ++s) {
      SG_BUSY_BEGIN
      if (s >= 1) {
        const SchurBatch B = d.sbatch[sg.bt0 + s - 1];
        const int npts = B.p1 - B.p0;
        const double* Xb = sh.X[(s - 1) & 1];
        const double* wsh = sh.w[(s - 1) % 3];
        const int4* pinf = sh.pinf[(s - 1) % 3];
        switch (cw) {
#define SG_SCHUR_CASE(W) \
          case W: schur_wave_batch<W>(acc, accr, Xb, wsh, pinf, npts, lane); break;
          SG_SCHUR_CASE(0) SG_SCHUR_CASE(1) SG_SCHUR_CASE(2) SG_SCHUR_CASE(3)
#if SG_SCHUR_CW > 4
          SG_SCHUR_CASE(4) SG_SCHUR_CASE(5) SG_SCHUR_CASE(6) SG_SCHUR_CASE(7)
#endif
#undef SG_SCHUR_CASE
        }
        SG_SSTAMP(42)
      }
      SG_BUSY_END
      __syncthreads();
      SG_SSTAMP(44)
    }
    mfma_drain();
    switch (cw) {
#define SG_SCHUR_CASE(W) \
      case W: schur_store<W>(acc, accr, slab, sg.ntw, lane); break;
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
#ifdef SG_SEG_STAMPS
  if (sstamp && lane == 0) {
    unsigned long long* ss = d.stamps + kSegStamp + 8 * seg;
    if (wave == 0) {
      ss[0] += __builtin_amdgcn_s_memtime() - t_wg;
      ss[1] += busy;
      ss[4] = sg.p0;
      ss[5] = sg.p1;
      ss[6] = nbt;
      ss[7] += 1;
    } else if (wave == kSchurCellWaves) {
      ss[2] += busy;
    } else if (wave == kSchurCellWaves + 1) {
      ss[3] += busy;
    }
  }
#endif
#undef SG_BUSY_BEGIN
#undef SG_BUSY_END
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
  const double xw = d.X[st->cur][4 * (size_t)p + 3];
  for (int o = obs_lo + tid; o < obs_hi; o += kSchurThreads) {
    const int b = d.frame_block[d.obs_frame[o]];
    if (b < 0) continue;
    double Jp[8], Jc[12];
    load_Jp_scaled(Jw, o, s4, Jp);
    load_Jc_scaled(d, Jw, o, b, xw, Jc);
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
    load_Jc_scaled(d, Jw, os, bs, xw, Jcs);
    load_Jc_scaled(d, Jw, ot, bt, xw, Jct);
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
// One element of a band tile of S: the four wave sums of its partials (in wave order), the wide-point
// accumulator and, on the assembling rank, the camera-only terms; written to S and returned.
__device__ __forceinline__ double s_tile_elem(const Dev& d, const double (&wsum)[4][256], int tid, size_t gi,
                                              double e_acc, int amode, int I, int Jb, int a, int c, double e_u,
                                              double e_fd, double e_si, double e_sj, double e_dg, double e_x,
                                              double radius) {
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
  return t;
}

// pre: the workgroup of tile (0, 0) also factors it (tile_factor, as k_chol_tiles' first owner would) into
// d.zpre: Z_0 = U_00^-T row-major [16][16], then a failure marker; k_chol_tiles (flags bit 4) starts from it, so
// the 16-pivot factor of D_0 is off the Cholesky's opening path (one rank, no free intrinsics: S is final here).
__global__ __launch_bounds__(256) void k_S_reduce(Dev d, int amode, int pre) {
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
        const int e = d.fd_pair[I * d.NB + Jb];   // 2 * residual + (frame a is block Jb)
        if (e >= 0) {
          const double* Xd = d.fd_X + 9 * (e >> 1);   // J_a J_b^T, rows: frame a's translation
          e_x = (e & 1) == 0 ? Xd[3 * (a - 3) + (c - 3)] : Xd[3 * (c - 3) + (a - 3)];
        }
      }
    }
    // the tile's padded list row: its first chunk of offsets goes out beside the count (no dependent round trip)
    const int j0 = wv * d.s_lstride, nlist = d.s_loff[wv];
    __shared__ double wsum[4][256];
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    constexpr int kSR = 8;
    int myoff = d.s_lidx[j0 + part + 4 * lane];
    for (int base = part; base < nlist; base += 4 * 64) {
      const int cnt = min(64, (nlist - base + 3) / 4);
      const int nxt = base + 4 * 64 < nlist ? d.s_lidx[j0 + base + 4 * 64 + 4 * lane] : 0;
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
      myoff = nxt;
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) wsum[part][lane + 64 * m] = s[m];
    __syncthreads();
    if (pre && rc == 0) {   // tile (0, 0), factored here (a workgroup-uniform branch: its barrier is safe)
      __shared__ double Dt[16 * kTLd], It[16 * kTLd], Yt[16], prt[2 * kCholNb];
      double t = 0.0;
      if (!done && live && up) t = s_tile_elem(d, wsum, tid, gi, e_acc, amode, I, Jb, a, c, e_u, e_fd, e_si, e_sj,
                                               e_dg, e_x, radius);
      if (!done && live && !up) {
        d.S[gi] = 0.0;
        if (d.nwide) d.S_wide[gi] = 0.0;
      }
      // as k_chol_tiles' tile_load pads past the system: 1 on the diagonal, 0 elsewhere
      const int ti = tid >> 4, tj = tid & 15;
      Dt[ti * kTLd + tj] = live ? (up ? t : 0.0) : (ti == tj ? 1.0 : 0.0);
      It[ti * kTLd + tj] = ti == tj ? 1.0 : 0.0;
      if (tid < 16) Yt[tid] = 0.0;
      __syncthreads();
      if (!done && tid < 64) {
        double ca[kCholNb];
        const bool bad = tile_factor(Dt, Yt, It, prt, ca);
        if (lane >= 16 && lane < 32)
#pragma unroll
          for (int r = 0; r < kCholNb; ++r) d.zpre[r * 16 + (lane - 16)] = ca[r];
        if (lane == 0) d.zpre[256] = bad ? 1.0 : 0.0;
      }
      return;
    }
    if (done || !live) return;
    if (!up) {
      d.S[gi] = 0.0;
      if (d.nwide) d.S_wide[gi] = 0.0;   // schur_pair_add also adds a diagonal block's lower half: keep it clean
      return;
    }
    s_tile_elem(d, wsum, tid, gi, e_acc, amode, I, Jb, a, c, e_u, e_fd, e_si, e_sj, e_dg, e_x, radius);
    return;
  }
  // rhs block I: one wave per 64-entry chunk of its partial list (in list order), lanes 0..5
  const int I = wv - d.nstile;
  // speculative linearization: clear block I of the candidate slot's wide-chunk camera accumulator before
  // k_update_lin adds to it (k_cam_reduce keeps the current slot's)
  if (d.spec && part == 1 && lane < kCamV) d.cam_wide[st->cur ^ 1][(size_t)I * kCamV + lane] = 0.0;
  const int j0 = I * d.r_lstride, j1 = j0 + d.r_loff[I];   // padded row: the first chunk needs no bound
  const int el = lane < 6 ? lane : 0;
  const int ei = 6 * I + el;
  const double e_acc = d.rhs[ei];
  const double e_si = amode != 0 ? d.scale_c[ei] : 0.0, e_g = amode != 0 ? d.camg[ei] : 0.0;
  __shared__ double rsum[4][6];
  constexpr int kSR = 32;
  double s = 0.0;
  int myoff = d.r_lidx[j0 + 64 * part + lane];
  for (int base = j0 + 64 * part; base < j1; base += 256) {
    const int cnt = min(64, j1 - base);
    const int nxt = base + 256 < j1 ? d.r_lidx[base + 256 + lane] : 0;
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

// Merged landmark-shard chain: the unpack of the summed band (k_S_pack's unpack) with k_cam_finalize mode 2 in
// the same launch — the LM diagonal (D^2 from the summed camera diagonal of the exchange tail, clamped, or the
// kept one when the step reuses it) divided by the radius added to each diagonal element as it is unpacked, and
// the minimizer bookkeeping on the summed tail in one extra workgroup (fin_merged_bookkeeping).  The bookkeeping
// changes no field the unpack reads (radius, reuse_diag, the diagonal clamps: LmState's concurrency contract).
__global__ __launch_bounds__(256) void k_S_unpack_fin(Dev d, const int32_t* panel_jend, const int32_t* off,
                                                      int npanel, const double* buf) {
  const int pk = blockIdx.x;
  if (pk == npanel + 1) {
    __shared__ double red[4];
    if (blockIdx.y == 0) fin_merged_bookkeeping(d, red);
    return;
  }
  const int n = d.n;
  const int stride = 256 * gridDim.y;
  if (pk == npanel) {
    double* xc = d.S + (size_t)n * n;
    for (int i = blockIdx.y * 256 + threadIdx.x; i < n; i += stride) xc[i] = buf[off[npanel] + i];
    return;
  }
  const LmState* st = d.st;
  const double radius = st->radius, min_diag = st->min_diag, max_diag = st->max_diag;
  const bool reuse = st->reuse_diag != 0;
  const double* tdg = d.xtail + 6 * d.NB;
  const int kb = pk * kCholNb, w = min(kCholNb, n - kb), width = panel_jend[pk] - kb;
  const int cnt = w * width;
  for (int e = blockIdx.y * 256 + threadIdx.x; e < cnt; e += stride) {
    const int r = e / width, c = e - r * width;
    const size_t gi = (size_t)(kb + r) * n + kb + c;
    double v = buf[off[pk] + e];
    if (r == c) {
      const int i = kb + r;
      double dg;
      if (!reuse) {
        const double s = d.scale_c[i];
        dg = fmin(fmax(s * s * tdg[i], min_diag), max_diag);
        d.diag_c[i] = dg;
      } else {
        dg = d.diag_c[i];
      }
      v += dg / radius;
    }
    d.S[gi] = v;
  }
}

// ------------------------------------------------------------------------------------------------
// host launchers (ba_launch.h)

void LaunchCamFinalizeK(hipStream_t s, const Dev& d, int mode, int decide) {
  hipLaunchKernelGGL(k_cam_finalize, dim3(1), dim3(256), 0, s, d, mode, decide);
}

void LaunchSchurK(int nseg, int nwide, int fin, hipStream_t s, const Dev& d) {
  hipLaunchKernelGGL(k_schur, dim3(nseg + (fin ? 1 : 0)), dim3(kSchurThreads), 0, s, d, fin);
  if (nwide) hipLaunchKernelGGL(k_schur_wide, dim3(nwide), dim3(kSchurThreads), 0, s, d);
}

void LaunchSUnpackFinK(dim3 grid, hipStream_t s, const Dev& d, const int32_t* panel_jend, const int32_t* off,
                       int npanel, const double* Spk) {
  hipLaunchKernelGGL(k_S_unpack_fin, dim3(grid.x + 1, grid.y), dim3(256), 0, s, d, panel_jend, off, npanel, Spk);
}

void LaunchSReduceK(int grid, hipStream_t s, const Dev& d, int amode, int pre) {
  hipLaunchKernelGGL(k_S_reduce, dim3(grid), dim3(256), 0, s, d, amode, pre);
}

void LaunchSPackK(dim3 grid, hipStream_t s, double* S, int n, const int32_t* panel_jend, const int32_t* off,
                  int npanel, double* Spk, int dir) {
  hipLaunchKernelGGL(k_S_pack, grid, dim3(256), 0, s, S, n, panel_jend, off, npanel, Spk, dir);
}

}  // namespace sg
