// schur_tiles.h — the matrix-core part of k_schur (ba_solver.hip): per segment window, the upper 16x16 tiles of
// S and the rhs held in v_mfma_f64_16x16x4f64 accumulators, one MFMA per (point, tile) with K = 4 (the rows of
// the point's whitened Jacobian E_p).  Device-only; shared with tools/schur_bench.hip.
#ifndef SG_SCHUR_TILES_H_
#define SG_SCHUR_TILES_H_

#include <hip/hip_runtime.h>

#include "ba_kernels.h"

namespace sg {

#ifndef SG_F64X4_DEFINED
#define SG_F64X4_DEFINED
typedef double f64x4 __attribute__((ext_vector_type(4)));   // v_mfma_f64_16x16x4f64 C/D operand
#endif

// Augmented slot order of a segment window: level c = 0 .. kSchurTW-1 holds the window tiles (0, c) .. (c, c),
// then the rhs tile of tile row c (E_c^T w in its column 0).  A point whose columns end in window tile jhi
// touches exactly the levels <= jhi: a prefix of schur_aug_base(jhi + 1) slots.  Wave W owns slots u = W + 4 s.
__host__ __device__ constexpr int schur_aug_base(int c) { return c * (c + 3) / 2; }
__host__ __device__ constexpr int schur_aug_c(int u) {
  int c = 0;
  while (schur_aug_base(c + 1) <= u) ++c;
  return c;
}
__host__ __device__ constexpr int schur_aug_r(int u) { return u - schur_aug_base(schur_aug_c(u)); }   // c + 1: rhs
// window tile (r, c), r <= c, in the segment slab's column-major upper order
__host__ __device__ constexpr int schur_tile_index(int r, int c) { return c * (c + 1) / 2 + r; }
__host__ __device__ constexpr int schur_tile_c(int t) {
  int c = 0;
  while ((c + 1) * (c + 2) / 2 <= t) ++c;
  return c;
}
__host__ __device__ constexpr int schur_tile_r(int t) { return t - schur_tile_c(t) * (schur_tile_c(t) + 1) / 2; }
// operand columns wave W reads
__host__ __device__ constexpr unsigned schur_need(int W) {
  unsigned m = 0;
  for (int u = W; u < kSchurAug; u += kSchurCWaves) {
    m |= 1u << schur_aug_c(u);
    if (schur_aug_r(u) <= schur_aug_c(u)) m |= 1u << schur_aug_r(u);
  }
  return m;
}

// The MFMAs run as inline asm (schur_chain.h): the compiler does not see them as MFMAs, so the hazards are ours.
// Readers of the accumulators must first call mfma_drain(); MFMA -> MFMA on the same accumulator is interlocked.
// wait states after the last asm MFMA before VALU / memory instructions read its accumulator
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 15\n\ts_nop 15" ::: "memory"); }

// One point: wave W runs the prefix of its slots below schur_aug_base(jhi + 1): the generated asm chain
// (schur_chain.h, tools/gen_schur_chain.py) entered at the offset that leaves exactly those slots, back to back.
// The point's operand tiles are 0 .. jhi of the window (zero outside its columns), so tiles with r below its
// first tile multiply zeros.
#include "schur_chain.h"
template <int W>
__device__ __forceinline__ void schur_mfma(f64x4 (&acc)[kSchurTPW], double (&accr)[kSchurTPW], const double (&X)[kSchurTW],
                                           double wop, int jhi) {
  const int nu = schur_aug_base(jhi + 1);
  SchurChain<W>::run(acc, accr, X, wop, (nu - W + kSchurCWaves - 1) / kSchurCWaves);
}

// Operands of point t of the batch (point table pv, one point per lane: {.., .., xoff | (jhi + 1) << 20, jhi};
// t >= npts: none): every operand column the wave may use, X_j[lane i + 16 k] = E_p[k][16 j + i] at xoff + 64 j
// (reads past the point's tiles land in the next point or the buffer's padding and feed only skipped slots), and
// the w operand of the rhs slots' v_mfma_f64_4x4x4_4b_f64 (B of block b, k x j at lane j + 4 b + 16 k: column 0 is
// w), read through the lane's own pointer wl into the point's 5-double w record {w_0 .. w_3, 0}: lanes with
// lane % 4 == 0 hold w_{lane / 16}, every other lane the zero (one VALU address per point, no select).  Every VALU instruction of an
// MFMA wave between two MFMAs costs ~16 cycles (tools/mfma_interleave.hip), so the point's table word is one
// v_readlane and the rest scalar.
template <unsigned kNeed>
__device__ __forceinline__ void schur_fetch(const double* Xb, const double* wl, const int4& pv, int t, int npts,
                                            int lane, double (&X)[kSchurTW], double& wop, int& jhi) {
  const int tt = min(t, npts - 1);
  const int v = __builtin_amdgcn_readlane(pv.z, tt);
  jhi = t < npts ? (v >> 20) - 1 : -1;
  const double* xp = Xb + (v & 0xfffff) + lane;
#pragma unroll
  for (int j = 0; j < kSchurTW; ++j)
    if ((kNeed >> j) & 1u) X[j] = xp[64 * j];
  wop = wl[5 * tt];
}
// The wave's work on one batch (whole wave active: the point table is read by v_readlane): the operands of
// point t + 1 are read before the MFMAs of point t.
template <int W>
__device__ __forceinline__ void schur_wave_batch(f64x4 (&acc)[kSchurTPW], double (&accr)[kSchurTPW], const double* Xb,
                                                 const double* wsh, const int4* pinf, int npts, int lane) {
  constexpr unsigned kNeed = schur_need(W);
  const int4 pv = pinf[min(lane, npts - 1)];   // npts <= 64
  const double* wl = wsh + ((lane & 3) == 0 ? (lane >> 4) : 4);
  double XA[kSchurTW], XB[kSchurTW];
#pragma unroll
  for (int j = 0; j < kSchurTW; ++j) XA[j] = XB[j] = 0.0;
  double wa, wb;
  int ha, hb;
  schur_fetch<kNeed>(Xb, wl, pv, 0, npts, lane, XA, wa, ha);
  for (int t = 0; t < npts; t += 2) {
    schur_fetch<kNeed>(Xb, wl, pv, t + 1, npts, lane, XB, wb, hb);
    schur_mfma<W>(acc, accr, XA, wa, ha);
    schur_fetch<kNeed>(Xb, wl, pv, t + 2, npts, lane, XA, wa, ha);
    schur_mfma<W>(acc, accr, XB, wb, hb);
  }
}

// Slab of a segment: its ntw (ntw + 1) / 2 window tiles (row-major 16x16, column-major upper order), then the
// rhs of its 16 ntw window columns.  The accumulators must be drained (mfma_drain) first.
template <int W>
__device__ __forceinline__ void schur_store(const f64x4 (&acc)[kSchurTPW], const double (&accr)[kSchurTPW], double* slab,
                                            int ntw, int lane) {
  const int ntile = ntw * (ntw + 1) / 2;
#pragma unroll
  for (int S = 0; S < kSchurTPW; ++S) {
    const int u = W + kSchurCWaves * S;
    if (u >= kSchurAug) break;
    const int c = schur_aug_c(u), r = schur_aug_r(u);
    if (c >= ntw) continue;
    if (r <= c) {
      double* t = slab + 256 * schur_tile_index(r, c) + lane;   // element (lk + 4 q, li) at 16 lk + li + 64 q
#pragma unroll
      for (int q = 0; q < 4; ++q) t[64 * q] = -acc[S][q];
    } else if ((lane & 3) == 0) {
      // E_c^T w (the 4 x 4 x 4 MFMA's D, block b row i column j at lane j + 4 b + 16 i): column 0, window row
      // 16 c + 4 b + i
      slab[256 * ntile + 16 * c + 4 * ((lane >> 2) & 3) + (lane >> 4)] = -accr[S];
    }
  }
}

}  // namespace sg

#endif  // SG_SCHUR_TILES_H_
