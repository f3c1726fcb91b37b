// Development microbenchmark (not part of the library): cycles of one 16x16 diagonal-tile factorisation with
// the identity (lanes 16-31) and the rhs (lane 32) as augmented columns — k_chol_tiles' critical step — one
// wave, variants side by side, outputs (Z = U^-T columns, z = U^-T y) compared with V0 on the host.
//   V0  the library's tile_factor: two pivots per LDS broadcast
//   V1  one pivot at a time, row broadcast by v_readlane (uniform SGPR multipliers, no LDS in the loop)
//   V2  V1 with the next pivot's column updated (and broadcast) first
//   V3  two pivots per step by v_readlane: rows j and j+1 broadcast together, pivot j+1 derived redundantly
// Also a second wave on the same SIMD issuing f64 MFMAs (the owner's SIMD mate in k_chol_tiles) when
// `mate` is set.  Build: hipcc --offload-arch=gfx950 -O3 tools/factor_bench2.hip -o tools/factor_bench2
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kNb = 16;
constexpr int kLd = 17;
typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double rsq_nr1(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  const double e = fma(-(h * y), y, 0.5);
  return fma(y, e, y);
}
__device__ __forceinline__ int opaque_lane() {
  int v = __lane_id();
  asm volatile("v_mov_b32 %0, %0" : "+v"(v));
  return v;
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// lanes 0-15 columns of D (upper, lower part zero), 16-31 identity, 32 rhs, others zero
__device__ __forceinline__ void load_cols(const double* D, const double* Id, const double* Yk, double (&ca)[16]) {
  const int lane = opaque_lane();
  const int c = lane & 15;
  const bool isy = lane == 32;
  const double* b0 = isy ? Yk : ((lane >= 16 && lane < 32) ? Id + c : D + c);
  const int rs = isy ? 1 : kLd;
#pragma unroll
  for (int r = 0; r < kNb; ++r) ca[r] = (lane < 33) ? b0[r * rs] : 0.0;
}

__device__ __forceinline__ bool factor_v0(double* prw, double (&ca)[16]) {
  const int lane = opaque_lane();
  bool bad = false;
  double u0[kNb], u1[kNb];
  double* prw2 = prw + kNb;
  if (lane < kNb) {
    prw[lane] = ca[0];
    prw2[lane] = ca[1];
  }
#pragma unroll
  for (int r = 0; r < kNb; ++r) {
    u0[r] = prw[r];
    u1[r] = prw2[r];
  }
#pragma unroll
  for (int j = 0; j < kNb; j += 2) {
    const double p0 = u0[j];
    bad |= !(p0 > 0.0);
    const double i0 = rsq_nr1(p0);
    const double r0 = i0 * i0;
    const double w1 = u0[j + 1] * r0;
    double v1[kNb];
#pragma unroll
    for (int r = j + 1; r < kNb; ++r) v1[r] = fma(-w1, u0[r], u1[r]);
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
    if (j + 2 < kNb) {
      ca[j + 2] = fma(-v1[j + 2], t1, fma(-u0[j + 2], t0, ca[j + 2]));
      ca[j + 3] = fma(-v1[j + 3], t1, fma(-u0[j + 3], t0, ca[j + 3]));
      if (lane < kNb) {
        prw[lane] = ca[j + 2];
        prw2[lane] = ca[j + 3];
      }
    }
#pragma unroll
    for (int r = j + 4; r < kNb; ++r) ca[r] = fma(-v1[r], t1, fma(-u0[r], t0, ca[r]));
#pragma unroll
    for (int r = j; r < kNb; ++r) asm volatile("" : "+v"(ca[r]));
    if (j + 2 < kNb) {
#pragma unroll
      for (int r = j + 2; r < kNb; ++r) {
        u0[r] = prw[r];
        u1[r] = prw2[r];
      }
    }
  }
  return bad;
}

// V1: row j of U = (lane r's ca[j]) * rsq(pivot), broadcast by readlane
__device__ __forceinline__ bool factor_v1(double (&ca)[16]) {
  bool bad = false;
#pragma unroll
  for (int j = 0; j < kNb; ++j) {
    const double piv = readlane_d(ca[j], j);
    bad |= !(piv > 0.0);
    const double inv = rsq_nr1(piv);
    ca[j] *= inv;
#pragma unroll
    for (int r = j + 1; r < kNb; ++r) ca[r] = fma(-readlane_d(ca[j], r), ca[j], ca[r]);
  }
  return bad;
}

// V2: unscaled row broadcast (readlane of the raw row j), the next pivot's column first
__device__ __forceinline__ bool factor_v2(double (&ca)[16]) {
  bool bad = false;
  double piv = readlane_d(ca[0], 0);
#pragma unroll
  for (int j = 0; j < kNb; ++j) {
    bad |= !(piv > 0.0);
    const double inv = rsq_nr1(piv);
    const double rj = inv * inv;
    const double aj = ca[j];
    const double t = aj * rj;
    ca[j] = aj * inv;
    if (j + 1 < kNb) {
      const double a1 = readlane_d(aj, j + 1);
      ca[j + 1] = fma(-a1, t, ca[j + 1]);
      piv = readlane_d(ca[j + 1], j + 1);
#pragma unroll
      for (int r = j + 2; r < kNb; ++r) ca[r] = fma(-readlane_d(aj, r), t, ca[r]);
    }
  }
  return bad;
}

// V3: two pivots per step; raw rows j and j+1 broadcast together (readlane), pivot j+1's row derived by every
// lane from them (uniform arithmetic), then both eliminations on the lane's own column
__device__ __forceinline__ bool factor_v3(double (&ca)[16]) {
  bool bad = false;
#pragma unroll
  for (int j = 0; j < kNb; j += 2) {
    double a[kNb], b[kNb];   // raw rows j and j+1 (columns >= j / >= j+1), uniform
#pragma unroll
    for (int r = j; r < kNb; ++r) a[r] = readlane_d(ca[j], r);
#pragma unroll
    for (int r = j + 1; r < kNb; ++r) b[r] = readlane_d(ca[j + 1], r);
    const double p0 = a[j];
    bad |= !(p0 > 0.0);
    const double i0 = rsq_nr1(p0);
    const double r0 = i0 * i0;
    const double w = a[j + 1] * r0;           // multiplier of row j in row j+1
    const double p1 = fma(-w, a[j + 1], b[j + 1]);
    bad |= !(p1 > 0.0);
    const double i1 = rsq_nr1(p1);
    const double r1 = i1 * i1;
    // own column: rows j, j+1
    const double cj = ca[j];
    const double t0 = cj * r0;
    ca[j] = cj * i0;
    const double cj1 = fma(-a[j + 1], t0, ca[j + 1]);
    const double t1 = cj1 * r1;
    ca[j + 1] = cj1 * i1;
#pragma unroll
    for (int r = j + 2; r < kNb; ++r) {
      const double br = fma(-w, a[r], b[r]);   // row j+1 after pivot j (uniform)
      ca[r] = fma(-br, t1, fma(-a[r], t0, ca[r]));
    }
  }
  return bad;
}

__device__ __forceinline__ f64x4 mfma_chain(f64x4 c, double a, double b, int n) {
  for (int i = 0; i < n; ++i) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  return c;
}

template <int V>
__global__ __launch_bounds__(128) void k_bench(const double* Dg, const double* Yg, double* out,
                                               unsigned long long* cyc, int iters, int mate) {
  __shared__ double D[kNb * kLd], Id[kNb * kLd];
  __shared__ double Y[kNb];
  __shared__ double prw[2 * kNb];
  const int tid = threadIdx.x;
  for (int i = tid; i < kNb * kLd; i += blockDim.x) {
    D[i] = Dg[i];
    Id[i] = (i / kLd == i % kLd) ? 1.0 : 0.0;
  }
  if (tid < kNb) Y[tid] = Yg[tid];
  __syncthreads();
  if (tid >= 64) {
    // the SIMD mate (wave 1 of a 2-wave workgroup lands on another SIMD; kept only as an option)
    if (mate) {
      f64x4 c = {0, 0, 0, 0};
      c = mfma_chain(c, 1e-3, 1e-3, 64 * iters);
      if (c[0] == 12345.0) out[0] = c[1];
    }
    return;
  }
  const int lane = tid;
  double ca[16];
  bool bad = false;
  unsigned long long t0 = 0;
  for (int it = 0; it <= iters; ++it) {
    if (it == 1) t0 = __builtin_amdgcn_s_memtime();
    load_cols(D, Id, Y, ca);
    if (V == 0) bad |= factor_v0(prw, ca);
    if (V == 1) bad |= factor_v1(ca);
    if (V == 2) bad |= factor_v2(ca);
    if (V == 3) bad |= factor_v3(ca);
    if (lane == 63) D[kNb * kLd - 1] = D[kNb * kLd - 1] + 0.0 * ca[15];   // ordering: one result feeds the next load
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[V] = (t1 - t0) / iters;
  for (int r = 0; r < kNb; ++r) out[(V * 64 + lane) * kNb + r] = ca[r];
  if (lane == 0 && bad) cyc[8 + V] = 1;
}

int main() {
  double hD[kNb * kLd] = {}, hY[kNb];
  srand(7);
  double B[kNb][kNb];
  for (int i = 0; i < kNb; ++i)
    for (int j = 0; j < kNb; ++j) B[i][j] = (rand() / (double)RAND_MAX) - 0.5;
  for (int i = 0; i < kNb; ++i) {
    hY[i] = (rand() / (double)RAND_MAX) - 0.5;
    for (int j = 0; j < kNb; ++j) {
      double s = (i == j) ? 4.0 : 0.0;
      for (int k = 0; k < kNb; ++k) s += B[i][k] * B[j][k];
      hD[i * kLd + j] = (i <= j) ? s : 0.0;   // upper triangle, lower zeroed
    }
  }
  double *dD, *dY, *dout;
  unsigned long long* dc;
  CHECK(hipMalloc(&dD, sizeof(hD)));
  CHECK(hipMalloc(&dY, sizeof(hY)));
  CHECK(hipMalloc(&dout, 8 * 64 * kNb * 8));
  CHECK(hipMalloc(&dc, 16 * 8));
  CHECK(hipMemcpy(dD, hD, sizeof(hD), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dY, hY, sizeof(hY), hipMemcpyHostToDevice));
  for (int mate = 0; mate < 2; ++mate) {
    CHECK(hipMemset(dc, 0, 16 * 8));
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(k_bench<0>, dim3(1), dim3(mate ? 128 : 64), 0, 0, dD, dY, dout, dc, 200, mate);
      hipLaunchKernelGGL(k_bench<1>, dim3(1), dim3(mate ? 128 : 64), 0, 0, dD, dY, dout, dc, 200, mate);
      hipLaunchKernelGGL(k_bench<2>, dim3(1), dim3(mate ? 128 : 64), 0, 0, dD, dY, dout, dc, 200, mate);
      hipLaunchKernelGGL(k_bench<3>, dim3(1), dim3(mate ? 128 : 64), 0, 0, dD, dY, dout, dc, 200, mate);
    }
    CHECK(hipDeviceSynchronize());
    unsigned long long hc[16];
    static double ho[8 * 64 * kNb];
    CHECK(hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost));
    for (int v = 0; v < 4; ++v) {
      double md = 0.0;
      for (int lane = 16; lane <= 32; ++lane)
        for (int r = 0; r < kNb; ++r)
          md = fmax(md, fabs(ho[(v * 64 + lane) * kNb + r] - ho[(0 * 64 + lane) * kNb + r]));
      printf("mate=%d V%d  %6llu cycles/factor   bad=%llu   max|Z,z - V0| = %.3g\n", mate, v, hc[v], hc[8 + v], md);
    }
  }
  return 0;
}
