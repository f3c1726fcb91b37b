// ba_tile.h — the 16x16 diagonal-tile factorisation shared by k_chol_tiles (ba_chol.hip) and k_S_reduce
// (ba_schur.hip, which factors the first diagonal tile as it assembles it, so the Cholesky starts from Z_0).
#ifndef SG_BA_TILE_H_
#define SG_BA_TILE_H_
#include "ba_kernels.h"

namespace sg {

constexpr int kTLd = 17;                       // LDS pitch of a 16 x 16 tile

// 1/sqrt(x): v_rsq_f64 and one Newton step in FMA form, y (1.5 - x y^2 / 2) (relative error ~1e-14, far
// inside the solver's parity tolerances; the pivot chain of the panel factorisation runs through it).
__device__ __forceinline__ double rsq_nr1(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  const double e = fma(-(h * y), y, 0.5);
  return fma(y, e, y);
}

// The lane id through an opaque move: comparisons against it inside a loop are not hoisted out as
// loop-invariant 64-bit lane masks (which would otherwise pile up in SGPRs and spill).
__device__ __forceinline__ int opaque_lane() {
  int v = __lane_id();
  asm volatile("v_mov_b32 %0, %0" : "+v"(v));
  return v;
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

}  // namespace sg

#endif  // SG_BA_TILE_H_
