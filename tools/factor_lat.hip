// factor_lat.hip — diagnostic: latency of one 16x16 diagonal-tile factorisation in a lone wave (no SIMD mate,
// no barrier), for the k_chol_tiles factor (tile_factor: two pivots per LDS broadcast), its generalisation to G
// pivots per broadcast (tile_factor_g<G>: G = 2 is bitwise tile_factor; G = 4 / 8 derive more pivot rows per lane)
// and the register form (tile_factor_mfma).  tile_factor is copied from slam-robot_amd/csrc/ba_chol.hip (keep in
// sync by hand; tool only).  Round 5: profiles/r5_factor_pivots_per_broadcast.log.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/factor_lat.hip -o tools/factor_lat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kCholNb = 16;
constexpr int kTLd = 17;
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


// tile_factor with G pivots per LDS broadcast: every lane derives the group's later pivot rows itself (row
// k + 1 .. G - 1 updated by pivot k in registers), so the 16 pivots take 16 / G LDS round trips.  G = 2 is
// bitwise tile_factor.
template <int G>
__device__ __forceinline__ bool tile_factor_g(const double* D, const double* Yk, const double* Id, double* prw,
                                              double (&ca)[16]) {
  const int lane = opaque_lane();
  const int c = lane & 15;
  const bool isy = lane == 32;
  const double* b0 = isy ? Yk : ((lane >= 16 && lane < 32) ? Id + c : D + c);
  const int rs = isy ? 1 : kTLd;
#pragma unroll
  for (int r = 0; r < kCholNb; ++r) ca[r] = b0[r * rs];
  bool bad = false;
  double u[G * kCholNb];
  if (lane < kCholNb) {
#pragma unroll
    for (int g = 0; g < G; ++g) prw[kCholNb * g + lane] = ca[g];
  }
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int r = g; r < kCholNb; ++r) u[kCholNb * (g) + r] = prw[kCholNb * g + r];
#pragma unroll
  for (int j = 0; j < kCholNb; j += G) {
    double rr[G], ii[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const double p = u[kCholNb * (k) + j + k];
      bad |= !(p > 0.0);
      ii[k] = rsq_nr1(p);
      rr[k] = ii[k] * ii[k];
#pragma unroll
      for (int g = k + 1; g < G; ++g) {
        const double w = u[kCholNb * (k) + j + g] * rr[k];
#pragma unroll
        for (int r = j + g; r < kCholNb; ++r) u[kCholNb * (g) + r] = fma(-w, u[kCholNb * (k) + r], u[kCholNb * (g) + r]);
      }
    }
    // this lane's column: the group's rows final, the next group's rows first (their broadcast goes out),
    // then the rest
    double t[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const double a = ca[j + k];
      t[k] = a * rr[k];
      ca[j + k] = a * ii[k];
#pragma unroll
      for (int r = j + k + 1; r < j + G; ++r) ca[r] = fma(-u[kCholNb * (k) + r], t[k], ca[r]);
    }
    if (j + G < kCholNb) {
#pragma unroll
      for (int r = j + G; r < j + 2 * G; ++r)
#pragma unroll
        for (int k = 0; k < G; ++k) ca[r] = fma(-u[kCholNb * (k) + r], t[k], ca[r]);
      if (lane < kCholNb) {
#pragma unroll
        for (int g = 0; g < G; ++g) prw[kCholNb * g + lane] = ca[j + G + g];
      }
    }
#pragma unroll
    for (int r = j + 2 * G; r < kCholNb; ++r)
#pragma unroll
      for (int k = 0; k < G; ++k) ca[r] = fma(-u[kCholNb * (k) + r], t[k], ca[r]);
#pragma unroll
    for (int r = j; r < kCholNb; ++r) asm volatile("" : "+v"(ca[r]));
    if (j + G < kCholNb) {
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int r = 0; r < kCholNb; ++r)   // (the whole row: a constant trip count unrolls; r < j + G + g is dead)
          if (r >= j + G + g) u[kCholNb * (g) + r] = prw[kCholNb * g + r];
    }
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


template <int mode>
__global__ __launch_bounds__(64) void k_lat(const double* Sg, const double* yg, int reps, double* out,
                                             unsigned long long* cyc, double* res) {
  __shared__ double Dw[16 * kTLd], Yw[16], Id[16 * kTLd], prw[16 * 8];
  const int lane = threadIdx.x, li = lane & 15, lk = lane >> 4;
  for (int i = lane; i < 16 * kTLd; i += 64) {
    Id[i] = (i / kTLd == i % kTLd) ? 1.0 : 0.0;
    const int r = i / kTLd, c = i % kTLd;
    Dw[i] = (c < 16 && r <= c) ? Sg[r * 16 + c] : 0.0;
  }
  if (lane < 16) Yw[lane] = yg[lane];
  __syncthreads();
  f64x4 D;
  for (int q = 0; q < 4; ++q) D[q] = Sg[(lk + 4 * q) * 16 + li];
  double acc = 0.0;
  bool bad = false;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    if constexpr (mode == 0 || mode >= 2) {
      double ca[16];
      if constexpr (mode == 0) bad |= tile_factor(Dw, Yw, Id, prw, ca);
      else bad |= tile_factor_g<mode>(Dw, Yw, Id, prw, ca);
      acc += ca[15];
      if (r == 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) res[16 * lane + i] = ca[i];
      }
      asm volatile("" ::: "memory");
    } else {
      double ys = yg[li] + acc * 1e-300;
      f64x4 Zt;
      bad |= tile_factor_mfma(D, ys, Zt, li, lk);
      acc += Zt[3] + ys;
      D[0] += acc * 1e-300;   // a dependence between repetitions
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = acc + (bad ? 1.0 : 0.0);
  if (lane == 0) *cyc = t1 - t0;
}

int main() {
  std::vector<double> S(256), y(16);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double v = 0.0;
      for (int k = 0; k < 16; ++k) v += std::sin(1.0 + i * 17 + k) * std::sin(1.0 + j * 17 + k);
      S[i * 16 + j] = v + (i == j ? 16.0 : 0.0);
    }
  for (int i = 0; i < 16; ++i) y[i] = std::cos(i);
  double *dS, *dy, *dout;
  unsigned long long* dc;
  hipMalloc(&dS, 256 * 8); hipMalloc(&dy, 128); hipMalloc(&dout, 64 * 8); hipMalloc(&dc, 8);
  hipMemcpy(dS, S.data(), 256 * 8, hipMemcpyHostToDevice);
  hipMemcpy(dy, y.data(), 128, hipMemcpyHostToDevice);
  const int reps = 2000;
  double* dres;
  hipMalloc(&dres, 64 * 16 * 8);
  std::vector<double> ref(64 * 16), got(64 * 16);
  const int modes[5] = {0, 2, 4, 8, 1};
  for (int mode : modes) {
    auto kf = mode == 0 ? k_lat<0> : mode == 1 ? k_lat<1> : mode == 2 ? k_lat<2> : mode == 4 ? k_lat<4> : k_lat<8>;
    hipLaunchKernelGGL(kf, dim3(1), dim3(64), 0, 0, dS, dy, 10, dout, dc, dres);
    hipLaunchKernelGGL(kf, dim3(1), dim3(64), 0, 0, dS, dy, reps, dout, dc, dres);
    unsigned long long c = 0;
    hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
    hipMemcpy(got.data(), dres, 64 * 16 * 8, hipMemcpyDeviceToHost);
    if (mode == 0) ref = got;
    double md = 0.0;
    int neq = 0;
    for (int l = 0; l < 33; ++l)
      for (int i = 0; i < 16; ++i) {
        const double a = ref[16 * l + i], b = got[16 * l + i];
        md = std::fmax(md, std::fabs(a - b) / std::fmax(1e-300, std::fabs(a)));
        neq += a != b;
      }
    if (mode == 1)
      std::printf("tile_factor_mfma: %.0f cycles per 16x16 factorisation (lone wave)\n", (double)c / reps);
    else
      std::printf("%s G=%d: %.0f cycles per 16x16 factorisation (lone wave); vs tile_factor: %d of 528 differ, "
                  "max rel %.2e\n", mode == 0 ? "tile_factor (LDS)" : "tile_factor_g", mode == 0 ? 2 : mode,
                  (double)c / reps, neq, md);
  }
  return 0;
}
