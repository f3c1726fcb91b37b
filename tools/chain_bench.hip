// chain_bench.hip — diagnostic (round 6): the k_chol_tiles owner's per-phase chain in isolation.  One workgroup of
// 8 waves (as the kernel); wave 0 runs NK phases of the owner's chain: the TRSM of its row-K tile with Z_K from the
// LDS ring, the U post, the diagonal update, then tile_diag (the diagonal tile to LDS, the rhs sum, the 16-pivot
// factor, the Z / z posts), one LDS barrier per phase; the other waves only meet the barriers (mode 0) or stay
// off the SIMD (mode 1: one-wave workgroup).  s_memtime stamps per part.  The device helpers are copies of
// slam-robot_amd/csrc/ba_chol.hip's (tool only: keep in sync by hand).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/chain_bench.hip -o tools/chain_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kCholNb = 16;
constexpr int kTLd = 17;
constexpr int kTB = 8;

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
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ f64x4 mfma_f64_k16(const double (&a)[4], const f64x4& b, f64x4 c) {
#pragma unroll
  for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], c, 0, 0, 0);
  return c;
}
__device__ __forceinline__ double sum_rows4(double v) {
  auto a = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
  auto b = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
  const double w = __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
  auto c = __builtin_amdgcn_permlane16_swap(__double2loint(w), __double2loint(w), false, false);
  auto e = __builtin_amdgcn_permlane16_swap(__double2hiint(w), __double2hiint(w), false, false);
  return __hiloint2double(e[0], c[0]) + __hiloint2double(e[1], c[1]);
}
struct TileShared {
  double Zs[4][16 * kTLd];
  double zK[4][16];
  double Ur[2][kTB - 1][256];
  double Dw[16 * kTLd];
  double Yw[16];
  double prw[2 * kCholNb];
  int fail, tmo, uflag;
  int simd[kTB];
  double Id[16 * kTLd];
};

__device__ __forceinline__ bool tile_factor(const double* D, const double* Yk, const double* Id, double* prw,
                                            double (&ca)[16]) {
  const int lane = opaque_lane();
  const int c = lane & 15;
  const bool isy = lane == 32;
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

__device__ __forceinline__ bool tile_diag(const f64x4& D, double ypart, TileShared& sh, int K, int lane, int li, int lk) {
#pragma unroll
  for (int q = 0; q < 4; ++q) sh.Dw[(lk + 4 * q) * kTLd + li] = (lk + 4 * q <= li) ? D[q] : 0.0;
  const double ys = sum_rows4(ypart);
  if (lk == 0) sh.Yw[li] = ys;
  double ca[kCholNb];
  const bool bad = tile_factor(sh.Dw, sh.Yw, sh.Id, sh.prw, ca);
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

#define STAMP(slot)                                                  \
  {                                                                  \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();    \
    acc[slot] += now_ - last;                                        \
    last = now_;                                                     \
  }

// mode 0: the full chain; mode 2: the factor alone on a posted tile (tile_factor, as tools/factor_lat.hip)
template <int kMode>
__global__ __launch_bounds__(512) void k_chain(const double* Ain, int NK, unsigned long long* out, double* sink) {
  __shared__ TileShared sh;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  for (int i = tid; i < 16 * kTLd; i += blockDim.x) {
    sh.Id[i] = (i / kTLd == i % kTLd) ? 1.0 : 0.0;
    for (int k = 0; k < 4; ++k) sh.Zs[k][i] = (i / kTLd == i % kTLd) ? 0.25 : 0.0;
    sh.Dw[i] = (i / kTLd == i % kTLd) ? 16.0 : 0.01;
  }
  for (int i = tid; i < 64; i += blockDim.x) sh.zK[i >> 4][i & 15] = 0.1;
  __syncthreads();
  unsigned long long acc[8] = {}, last = __builtin_amdgcn_s_memtime();
  f64x4 A1, D0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    A1[q] = Ain[lane + 64 * q];
    D0[q] = Ain[256 + lane + 64 * q];
  }
  double ypart = 0.01 * lane;
  bool bad = false;
  double keep = 0.0;
  for (int K = 0; K < NK; ++K) {
    if (wave == 0) {
      STAMP(0)
      if (kMode == 0) {
        const double* Zs = sh.Zs[K & 3];
        const f64x4 zero = {0.0, 0.0, 0.0, 0.0};
        double za[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) za[s] = Zs[li * kTLd + 4 * s + lk];
        const f64x4 U = mfma_f64_k16(za, A1, zero);
        double* ur = sh.Ur[K & 1][0];
#pragma unroll
        for (int q = 0; q < 4; ++q) ur[q * 64 + lane] = U[q];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&sh.uflag, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const double* zk = sh.zK[K & 3];
        double yp = ypart;
#pragma unroll
        for (int q = 0; q < 4; ++q) yp = fma(-U[q], zk[lk + 4 * q], yp);
        STAMP(1)
        double a[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = -U[s];
        const f64x4 D = mfma_f64_k16(a, U, D0);
        STAMP(2)
        bad |= tile_diag(D, yp, sh, K + 1, lane, li, lk);
        STAMP(3)
      } else {
        double ca[16];
        bad |= tile_factor(sh.Dw, sh.Yw, sh.Id, sh.prw, ca);
        keep += ca[15];
        STAMP(3)
      }
    }
    lds_barrier();
    if (wave == 0) STAMP(4)
  }
  if (tid == 0)
    for (int s = 0; s < 8; ++s) out[s] = acc[s];
  if (bad || keep == 12345.0) sink[tid] = keep;
}

int main() {
  const int NK = 2000;
  std::vector<double> A(512);
  for (int i = 0; i < 512; ++i) A[i] = (i < 256 ? 0.01 : 0.0) * ((i * 37) % 11 - 5) + (i >= 256 && ((i & 15) == (((i & 63) >> 4) + 4 * ((i - 256) >> 6))) ? 16.0 : 0.0);
  double *dA, *dS;
  unsigned long long* dO;
  hipMalloc(&dA, 512 * sizeof(double));
  hipMalloc(&dS, 512 * sizeof(double));
  hipMalloc(&dO, 8 * sizeof(unsigned long long));
  hipMemcpy(dA, A.data(), 512 * sizeof(double), hipMemcpyHostToDevice);
  const char* names[] = {"phase start -> after TRSM + U post (1)", "diagonal update (2)", "tile_diag: D to LDS, rhs sum, factor, posts (3)",
                         "barrier (4)"};
  for (int mode : {0, 2})
    for (int waves : {8, 1}) {
      for (int rep = 0; rep < 2; ++rep) {
        if (mode == 0)
          hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64 * waves), 0, 0, dA, NK, dO, dS);
        else
          hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64 * waves), 0, 0, dA, NK, dO, dS);
      }
      hipDeviceSynchronize();
      unsigned long long o[8];
      hipMemcpy(o, dO, sizeof(o), hipMemcpyDeviceToHost);
      std::printf("mode %s, %d waves: cycles per phase:", mode == 0 ? "full owner chain" : "factor alone", waves);
      unsigned long long tot = 0;
      for (int s = 1; s <= 4; ++s) tot += o[s];
      tot += o[0];
      for (int s = 1; s <= 4; ++s) std::printf("  [%s] %.0f", names[s - 1], (double)o[s] / NK);
      std::printf("  total %.0f\n", (double)tot / NK);
    }
  return 0;
}
