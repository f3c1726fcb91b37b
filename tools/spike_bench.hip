// spike_bench.hip — diagnostic (round 6, VERDICT r5 item 1b's gate): the two terms of the four-leaf dissection
// that DESIGN.md §5 could only model, measured on the device.
//   * A middle leaf's workgroup (the producer) runs the owner chain of each phase (TRSM, diagonal update and the
//     library's own 16-pivot tile_factor from ba_tile.h, as tools/chain_bench.hip) while its seven other waves
//     issue 16 trailing MFMAs each.  With posts (mode bit 1), every wave also stores one 16x16 tile per phase
//     (the row's W tiles and Z), the waves drain their stores, and wave 7 releases at agent scope and raises the
//     row's flag: the per-phase cost of handing every row to another workgroup.
//   * The spike workgroup (mode bit 2) follows the posts: per row K it waits for the flag, then each of waves 0-6
//     (one tile column of the separator border) forms v_K = A - sum_{d=1..7} W_{K-d,K}^T v_{K-d} (28 MFMAs) and
//     w_K = Z_K v_K (4), posts w_K to LDS, and the eight waves form the 28 upper tiles of the separator update
//     sum w_K^T w_K (16 MFMAs on waves 0-6).
// Realtime stamps (s_memrealtime, 100 MHz, one clock for both workgroups) per row: the producer's pace with and
// without posts, the spike chain's pace and its lag behind the producer.  Numbers only; no results are checked.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -Islam-robot_amd/csrc tools/spike_bench.hip -o tools/spike_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "ba_tile.h"

using namespace sg;
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kWaves = 8;

__device__ __forceinline__ f64x4 mfma_k16(const double (&a)[4], const f64x4& b, f64x4 c) {
#pragma unroll
  for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], c, 0, 0, 0);
  return c;
}
__device__ __forceinline__ void lds_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

struct ProdShared {
  double Zs[4][16 * kTLd];
  double Dw[16 * kTLd];
  double Yw[16];
  double prw[2 * kCholNb];
  double Id[16 * kTLd];
};
struct SpikeShared {
  double w[kWaves][256];
};

// Wpost: [NK][8][256] tiles (slot 0 of row K: Z_{K+1}; slots 1..7: the row's W tiles); flag: rows posted.
template <int kMode>
__global__ __launch_bounds__(512) void k_spike(const double* Ain, double* Wpost, int* flag, int NK,
                                               unsigned long long* tprod, unsigned long long* tspike, double* sink) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  f64x4 A1, D0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    A1[q] = Ain[lane + 64 * q];
    D0[q] = Ain[256 + lane + 64 * q];
  }
  double keep = 0.0;
  if (blockIdx.x == 0) {
    __shared__ ProdShared sh;
    for (int i = tid; i < 16 * kTLd; i += blockDim.x) {
      sh.Id[i] = (i / kTLd == i % kTLd) ? 1.0 : 0.0;
      for (int k = 0; k < 4; ++k) sh.Zs[k][i] = (i / kTLd == i % kTLd) ? 0.25 : 0.0;
    }
    __syncthreads();
    f64x4 T = A1;
    bool bad = false;
    for (int K = 0; K < NK; ++K) {
      f64x4 post = A1;
      if (wave == 0) {
        // the owner chain: TRSM with Z_K, the diagonal update, the 16-pivot factor of the next diagonal
        const double* Zs = sh.Zs[K & 3];
        const f64x4 zero = {0.0, 0.0, 0.0, 0.0};
        double za[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) za[s] = Zs[li * kTLd + 4 * s + lk];
        const f64x4 U = mfma_k16(za, A1, zero);
        double a[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = -U[s];
        const f64x4 D = mfma_k16(a, U, D0);
#pragma unroll
        for (int q = 0; q < 4; ++q) sh.Dw[(lk + 4 * q) * kTLd + li] = (lk + 4 * q <= li) ? D[q] : 0.0;
        if (lane < 16) sh.Yw[lane] = 0.01 * lane;
        double ca[kCholNb];
        bad |= tile_factor(sh.Dw, sh.Yw, sh.Id, sh.prw, ca);
        double* Zn = sh.Zs[(K + 1) & 3];
        if (lane >= 16 && lane < 32)
#pragma unroll
          for (int r = 0; r < kCholNb; ++r) Zn[r * kTLd + (lane - 16)] = ca[r];
        post = D;
      } else {
        // the column waves' trailing updates (16 MFMAs each, the band's mean)
        double a[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = A1[s] * 1e-3;
#pragma unroll
        for (int r = 0; r < 4; ++r) T = mfma_k16(a, T, T);
        post = T;
      }
      if (kMode & 1) {
        double* dst = Wpost + ((size_t)K * kWaves + wave) * 256 + lane;
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[64 * q] = post[q];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // this wave's stores complete (vscnt 0)
      }
      lds_bar();
      if ((kMode & 1) && wave == kWaves - 1 && lane == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");       // the L2 write-back, off the chain wave
        __hip_atomic_store(flag, K + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (tid == 0) tprod[K] = rt();
    }
    keep = T[0] + (bad ? 1.0 : 0.0);
  } else {
    if (!(kMode & 2)) return;
    __shared__ SpikeShared ss;
    __shared__ int go;
    f64x4 v[7];
#pragma unroll
    for (int d = 0; d < 7; ++d) v[d] = {0.0, 0.0, 0.0, 0.0};
    f64x4 S[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) S[t] = {0.0, 0.0, 0.0, 0.0};
    if (kMode & 4) {
      // pipelined: row K's operands (the W tiles of rows K-1..K-7 and Z_K, posted by row K-1) are loaded during row
      // K-1's MFMAs, right after row K-1's flag; the separator update is left to one GEMM after the leaf
      double cw[7][4], cz[4], nw[7][4], nz[4];
      auto load_row = [&](double (&w)[7][4], double (&z)[4], int K) {
#pragma unroll
        for (int d = 1; d <= 7; ++d) {
          const int Kd = K - d >= 0 ? K - d : 0;
          const double* src = Wpost + ((size_t)Kd * kWaves + d) * 256 + lane;
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) w[d - 1][s2] = src[64 * s2];
        }
        const double* zs = Wpost + ((size_t)(K >= 1 ? K - 1 : 0) * kWaves) * 256 + lane;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) z[s2] = zs[64 * s2];
      };
      auto wait_flag = [&](int val) {
        if (tid == 0) {
          int spin = 0;
          while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < val && ++spin < (1 << 24))
            __builtin_amdgcn_s_sleep(1);
          go = spin;
        }
        lds_bar();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      };
      // two register buffers, the loop unrolled by two: row K computes from one while row K + 1's loads land in
      // the other (a copy between them would make the compiler wait for the loads inside the same row)
      auto step = [&](int K, double (&uw)[7][4], double (&uz)[4], double (&lw)[7][4], double (&lz)[4]) {
        if (K + 1 < NK) {
          wait_flag(K + 1);   // row K posted: row K + 1's operands are all out
          load_row(lw, lz, K + 1);
        }
        if (wave < 7) {
          f64x4 acc = A1;
#pragma unroll
          for (int d = 1; d <= 7; ++d) {
            double a[4];
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) a[s2] = -uw[d - 1][s2] * 1e-3;
            acc = mfma_k16(a, v[d - 1], acc);
          }
          double z[4];
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) z[s2] = uz[s2] * 1e-3;
          const f64x4 zero = {0.0, 0.0, 0.0, 0.0};
          const f64x4 w = mfma_k16(z, acc, zero);
#pragma unroll
          for (int d = 6; d >= 1; --d) v[d] = v[d - 1];
          v[0] = acc;
          S[0] += w;
        }
        if (tid == 0) tspike[K] = rt();
      };
      wait_flag(1);
      load_row(cw, cz, 0);
      for (int K = 0; K < NK; K += 2) {
        step(K, cw, cz, nw, nz);
        if (K + 1 < NK) step(K + 1, nw, nz, cw, cz);
      }
    } else
    for (int K = 0; K < NK; ++K) {
      if (tid == 0) {
        int spin = 0;
        while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= K && ++spin < (1 << 24))
          __builtin_amdgcn_s_sleep(1);
        go = spin;
      }
      lds_bar();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (wave < 7) {
        // v_K = A - sum_d W_{K-d,K}^T v_{K-d}; w_K = Z_K v_K (row K's slot 0)
        f64x4 acc = A1;
#pragma unroll
        for (int d = 1; d <= 7; ++d) {
          const int Kd = K - d >= 0 ? K - d : 0;
          const double* src = Wpost + ((size_t)Kd * kWaves + d) * 256 + lane;
          double a[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) a[s] = -src[64 * s] * 1e-3;
          acc = mfma_k16(a, v[d - 1], acc);
        }
        const double* zs = Wpost + ((size_t)K * kWaves) * 256 + lane;
        double z[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) z[s] = zs[64 * s] * 1e-3;
        const f64x4 zero = {0.0, 0.0, 0.0, 0.0};
        const f64x4 w = mfma_k16(z, acc, zero);
#pragma unroll
        for (int d = 6; d >= 1; --d) v[d] = v[d - 1];
        v[0] = acc;
#pragma unroll
        for (int q = 0; q < 4; ++q) ss.w[wave][lane + 64 * q] = w[q];
      }
      lds_bar();
      if (wave < 7) {
        // four of the 28 upper tiles of sum w^T w: wave c takes pairs 4c .. 4c + 3 (row-major over c1 <= c2)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int p = 4 * wave + t;
          int c1 = 0, rem = p;
          while (rem >= 7 - c1) {
            rem -= 7 - c1;
            ++c1;
          }
          const int c2 = c1 + rem;
          double a[4];
          f64x4 b;
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            a[s] = ss.w[c1][lane + 64 * s];
            b[s] = ss.w[c2][lane + 64 * s];
          }
          S[t] = mfma_k16(a, b, S[t]);
        }
      }
      lds_bar();
      if (tid == 0) tspike[K] = rt();
    }
    keep = S[0][0] + S[1][1] + S[2][2] + S[3][3] + v[0][0] + go;
  }
  if (keep == 12345.0) sink[tid] = keep;
}

template <int kMode>
static void run(const double* dA, double* dW, int* dF, int NK, unsigned long long* dP, unsigned long long* dS,
                double* dSink, std::vector<unsigned long long>& hp, std::vector<unsigned long long>& hs) {
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(dF, 0, sizeof(int));
    hipLaunchKernelGGL(k_spike<kMode>, dim3(kMode & 2 ? 2 : 1), dim3(64 * kWaves), 0, 0, dA, dW, dF, NK, dP, dS, dSink);
    hipDeviceSynchronize();
  }
  hipMemcpy(hp.data(), dP, NK * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  hipMemcpy(hs.data(), dS, NK * sizeof(unsigned long long), hipMemcpyDeviceToHost);
}

int main() {
  const int NKmax = 400;
  std::vector<double> A(512);
  for (int i = 0; i < 512; ++i)
    A[i] = (i < 256 ? 0.01 : 0.0) * ((i * 37) % 11 - 5) +
           (i >= 256 && ((i & 15) == (((i & 63) >> 4) + 4 * ((i - 256) >> 6))) ? 16.0 : 0.0);
  double *dA, *dW, *dSink;
  int* dF;
  unsigned long long *dP, *dS;
  hipMalloc(&dA, 512 * sizeof(double));
  hipMalloc(&dW, (size_t)NKmax * kWaves * 256 * sizeof(double));
  hipMalloc(&dSink, 512 * sizeof(double));
  hipMalloc(&dF, sizeof(int));
  hipMalloc(&dP, NKmax * sizeof(unsigned long long));
  hipMalloc(&dS, NKmax * sizeof(unsigned long long));
  hipMemcpy(dA, A.data(), 512 * sizeof(double), hipMemcpyHostToDevice);
  hipMemset(dW, 0, (size_t)NKmax * kWaves * 256 * sizeof(double));
  hipMemset(dS, 0, NKmax * sizeof(unsigned long long));
  for (int NK : {14, 35, 400}) {
    std::vector<unsigned long long> p0(NK), s0(NK), p1(NK), s1(NK), p3(NK), s3(NK);
    run<0>(dA, dW, dF, NK, dP, dS, dSink, p0, s0);
    run<1>(dA, dW, dF, NK, dP, dS, dSink, p1, s1);
    run<3>(dA, dW, dF, NK, dP, dS, dSink, p3, s3);
    std::vector<unsigned long long> p7(NK), s7(NK);
    run<7>(dA, dW, dF, NK, dP, dS, dSink, p7, s7);
    auto per = [&](const std::vector<unsigned long long>& t) { return 10.0 * (t[NK - 1] - t[0]) / (NK - 1); };   // ns
    std::printf("rows %3d: producer ns/phase  alone %.0f  with posts %.0f  with posts + spike wg %.0f | spike ns/row %.0f,"
                " lag at the last row %.0f ns (%.2f phases), first row %.0f ns\n",
                NK, per(p0), per(p1), per(p3), per(s3), 10.0 * ((double)s3[NK - 1] - (double)p3[NK - 1]),
                ((double)s3[NK - 1] - (double)p3[NK - 1]) * 10.0 / per(p3), 10.0 * ((double)s3[0] - (double)p3[0]));
    std::printf("rows %3d: pipelined spike wg (no per-row separator update): producer ns/phase %.0f, spike ns/row %.0f,"
                " lag at the last row %.0f ns (%.2f phases)\n",
                NK, per(p7), per(s7), 10.0 * ((double)s7[NK - 1] - (double)p7[NK - 1]),
                ((double)s7[NK - 1] - (double)p7[NK - 1]) * 10.0 / per(p7));
  }
  return 0;
}
