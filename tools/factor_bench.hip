// Development microbenchmark (not part of the library): cycles of one 16x16 diagonal-tile factorisation
// with the identity and the rhs as augmented columns (k_chol_tiles' critical step), one wave, variants side
// by side; the outputs (Z = U^-T columns, z = U^-T y) are compared on the host.
// Build: hipcc --offload-arch=gfx950 -O3 tools/factor_bench.hip -o tools/factor_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kNb = 16;
constexpr int kLd = 17;

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

// shared prologue: lanes 0-15 columns of D (upper), 16-31 identity, 32 rhs
__device__ __forceinline__ void load_cols(const double* D, const double* Yk, double (&ca)[16]) {
  const int lane = opaque_lane();
  const int c = lane & 15;
  const bool isy = lane == 32;
  const double* b0 = isy ? Yk : D + c;
  const int rs = isy ? 1 : kLd;
#pragma unroll
  for (int r = 0; r < kNb; ++r) ca[r] = b0[r * rs];
  unsigned keepbits = lane < 16 ? ((2u << c) - 1u) : (isy ? 0xFFFFu : 0u);
  unsigned onebits = (lane >= 16 && lane < 32) ? (1u << c) : 0u;
  asm volatile("" : "+v"(keepbits), "+v"(onebits));
  const unsigned long long kOneBits = 0x3FF0000000000000ull;
#pragma unroll
  for (int r = 0; r < kNb; ++r) {
    int km, om;
    asm volatile("v_bfe_i32 %0, %1, %2, 1" : "=v"(km) : "v"(keepbits), "n"(r));
    asm volatile("v_bfe_i32 %0, %1, %2, 1" : "=v"(om) : "v"(onebits), "n"(r));
    const unsigned long long b = (unsigned long long)__double_as_longlong(ca[r]);
    ca[r] = __longlong_as_double((long long)((b & (unsigned long long)(long long)km) |
                                             (kOneBits & (unsigned long long)(long long)om)));
  }
}

// V0: two pivots per LDS broadcast (the library's tile_factor)
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

// V1: one pivot at a time, row broadcast by v_readlane (no LDS in the loop)
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

// V2: one pivot at a time; the next pivot's column first (critical chain), readlane broadcasts
__device__ __forceinline__ bool factor_v2(double (&ca)[16]) {
  bool bad = false;
  double piv = readlane_d(ca[0], 0);
#pragma unroll
  for (int j = 0; j < kNb; ++j) {
    bad |= !(piv > 0.0);
    const double inv = rsq_nr1(piv);
    const double rj = inv * inv;
    // U[j][r] A[j][c] / A_jj form: t = A[j][c] / A_jj, update with the unscaled row value A[j][r]
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

template <int V>
__global__ __launch_bounds__(64) void k_bench(const double* Dg, const double* Yg, double* out,
                                              unsigned long long* cyc, int iters) {
  __shared__ double D[kNb * kLd];
  __shared__ double Y[kNb];
  __shared__ double prw[2 * kNb];
  const int lane = threadIdx.x;
  for (int i = lane; i < kNb * kLd; i += 64) D[i] = Dg[i];
  if (lane < kNb) Y[lane] = Yg[lane];
  __syncthreads();
  double ca[16];
  bool bad = false;
  unsigned long long t0 = 0;
  for (int it = 0; it <= iters; ++it) {
    if (it == 1) t0 = __builtin_amdgcn_s_memtime();
    load_cols(D, Y, ca);
    if (V == 0) bad |= factor_v0(prw, ca);
    if (V == 1) bad |= factor_v1(ca);
    if (V == 2) bad |= factor_v2(ca);
    // feed the result back (dependency across iterations): perturb nothing, just a ordering fence
    if (lane == 63) D[0] = D[0] + 0.0 * ca[15];
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
      hD[i * kLd + j] = s;
    }
  }
  double *dD, *dY, *dout;
  unsigned long long* dc;
  CHECK(hipMalloc(&dD, sizeof(hD)));
  CHECK(hipMalloc(&dY, sizeof(hY)));
  CHECK(hipMalloc(&dout, 4 * 64 * kNb * 8));
  CHECK(hipMalloc(&dc, 16 * 8));
  CHECK(hipMemset(dc, 0, 16 * 8));
  CHECK(hipMemcpy(dD, hD, sizeof(hD), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dY, hY, sizeof(hY), hipMemcpyHostToDevice));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_bench<0>, dim3(1), dim3(64), 0, 0, dD, dY, dout, dc, 200);
    hipLaunchKernelGGL(k_bench<1>, dim3(1), dim3(64), 0, 0, dD, dY, dout, dc, 200);
    hipLaunchKernelGGL(k_bench<2>, dim3(1), dim3(64), 0, 0, dD, dY, dout, dc, 200);
  }
  CHECK(hipDeviceSynchronize());
  unsigned long long hc[16];
  double ho[4 * 64 * kNb];
  CHECK(hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost));
  for (int v = 0; v < 3; ++v) {
    double md = 0.0;
    for (int lane = 16; lane <= 32; ++lane)
      for (int r = 0; r < kNb; ++r)
        md = fmax(md, fabs(ho[(v * 64 + lane) * kNb + r] - ho[(0 * 64 + lane) * kNb + r]));
    printf("V%d  %6llu cycles/factor   bad=%llu   max|Z,z - V0| = %.3g\n", v, hc[v], hc[8 + v], md);
  }
  return 0;
}
