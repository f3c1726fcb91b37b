// Latency microbenchmarks for the single-workgroup solver kernels (development tool, not part of the
// library): s_memtime cycles for an LDS round trip, a workgroup barrier, a global load, a dependent fp64
// FMA chain, v_readlane broadcasts and a wave reduction.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <int kCtrl>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), kCtrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), kCtrl, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_dd(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum_full(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x141>(v);
  v += dpp_d<0x140>(v);
  return (readlane_dd(v, 0) + readlane_dd(v, 16)) + (readlane_dd(v, 32) + readlane_dd(v, 48));
}

__global__ __launch_bounds__(512) void k_lat(const double* g, double* out, unsigned long long* t, int iters) {
  __shared__ double sh[1024];
  const int tid = threadIdx.x, lane = tid & 63;
  double acc = g[tid];
  sh[tid] = acc;
  __syncthreads();
  unsigned long long t0, t1;
  // 1. LDS write -> read round trip (one wave, dependent)
  t0 = __builtin_amdgcn_s_memtime();
  if (tid < 64) {
    for (int i = 0; i < iters; ++i) {
      sh[lane] = acc;
      acc = sh[(lane + 1) & 63] * 1.0000001;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[0] = (t1 - t0) / iters;
  __syncthreads();
  // 2. barrier (8 waves)
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) lds_barrier();
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[1] = (t1 - t0) / iters;
  // 3. global load latency (dependent chain)
  int idx = tid;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    const double v = g[idx];
    idx = ((int)v + idx + 1) & 1023;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[2] = (t1 - t0) / iters;
  acc += idx;
  // 4. dependent fp64 FMA chain
  double x = acc;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) x = fma(x, 1.0000001, 1e-9);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[3] = (t1 - t0) / (16 * iters);
  // 5. readlane broadcast + FMA chain
  double y = acc;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int lo = __builtin_amdgcn_readlane(__double2loint(y), k);
      const int hi = __builtin_amdgcn_readlane(__double2hiint(y), k);
      y = fma(__hiloint2double(hi, lo), 1e-9, y);
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[4] = (t1 - t0) / (16 * iters);
  // 6. wave reduction
  double z = acc;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) z = wave_sum(z) * 1e-3;
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[5] = (t1 - t0) / iters;
  // 7. fp64 rsq + 2 Newton
  double r = acc + 2.0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    double inv = __builtin_amdgcn_rsq(r);
    inv = inv * (1.5 - 0.5 * r * inv * inv);
    inv = inv * (1.5 - 0.5 * r * inv * inv);
    r = inv + 2.0;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[6] = (t1 - t0) / iters;
  // 8. LDS broadcast read of 16 doubles (8 x b128) after a write (one wave)
  double w = acc;
  t0 = __builtin_amdgcn_s_memtime();
  if (tid < 64) {
    for (int i = 0; i < iters; ++i) {
      if (lane < 16) sh[lane] = w;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 16; ++k) s += sh[k];
      w = s * 1e-3;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[7] = (t1 - t0) / iters;
  // 9. DPP wave reduction
  double q = acc + lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) q = wave_sum_full(q) * 1e-3 + lane;
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[8] = (t1 - t0) / iters;
  const double chk = wave_sum_full((double)lane);   // all lanes active; 2016 expected
  if (tid == 0) t[9] = (unsigned long long)chk;
  // 10. dependent v_mfma_f64_16x16x4f64 chain (one wave)
  typedef double f64x4 __attribute__((ext_vector_type(4)));
  f64x4 m = {acc, acc, acc, acc};
  const double ma = acc * 1e-9 + 1e-12, mb = acc + 1e-3;
  __syncthreads();
  t0 = __builtin_amdgcn_s_memtime();
  if (tid < 64) {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) m = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, m, 0, 0, 0);
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[10] = (t1 - t0) / (8 * iters);
  // 11. same chain, all 8 waves (two per SIMD) at once
  __syncthreads();
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) m = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, m, 0, 0, 0);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[11] = (t1 - t0) / (8 * iters);
  // 12. four independent accumulators, one wave (issue rate)
  f64x4 m1 = m, m2 = m, m3 = m;
  __syncthreads();
  t0 = __builtin_amdgcn_s_memtime();
  if (tid < 64) {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        m = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, m, 0, 0, 0);
        m1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, m1, 0, 0, 0);
        m2 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, m2, 0, 0, 0);
        m3 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, m3, 0, 0, 0);
      }
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[12] = (t1 - t0) / (8 * iters);
  // 13. LDS write then dependent 4 x ds_read_b64 (lane-dependent addresses) + use
  double v13 = acc;
  __syncthreads();
  t0 = __builtin_amdgcn_s_memtime();
  if (tid < 64) {
    for (int i = 0; i < iters; ++i) {
      sh[lane] = v13;
      v13 = (sh[(lane * 5) & 63] + sh[(lane * 7) & 63]) * 0.5 + (sh[(lane * 3) & 63] + sh[(lane * 11) & 63]) * 1e-9;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[13] = (t1 - t0) / iters;
  out[tid] = acc + x + y + z + r + w + q + m[0] + m[1] + m[2] + m[3] + m1[0] + m2[1] + m3[2] + v13;
}

int main() {
  double *g, *out;
  unsigned long long* t;
  CHECK(hipMalloc(&g, 1024 * 8));
  CHECK(hipMalloc(&out, 1024 * 8));
  CHECK(hipMalloc(&t, 16 * 8));
  CHECK(hipMemset(g, 0, 1024 * 8));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(512), 0, 0, g, out, t, 200);
    CHECK(hipDeviceSynchronize());
  }
  unsigned long long h[16];
  CHECK(hipMemcpy(h, t, 16 * 8, hipMemcpyDeviceToHost));
  const char* names[] = {"LDS write->read round trip", "8-wave LDS barrier", "global load (dependent)",
                         "fp64 FMA (dependent)", "readlane pair + FMA", "wave_sum (shfl_xor)",
                         "rsq + 2 Newton", "LDS write + 16 broadcast reads + adds",
                         "wave_sum_full (DPP)", "check: sum of lane ids (2016)",
                         "f64 MFMA 16x16x4 dependent (1 wave)", "f64 MFMA dependent (8 waves)",
                         "f64 MFMA 4 independent (1 wave)", "LDS write + 4 reads + use"};
  for (int i = 0; i < 14; ++i) printf("%-40s %6llu cycles\n", names[i], h[i]);
  return 0;
}
