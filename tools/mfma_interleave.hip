// Development microbenchmark (not part of the library): what other instructions of the same wave cost between
// back-to-back v_mfma_f64_16x16x4f64 on gfx950 (k_schur's MFMA waves run a per-point chain of ~5 MFMAs with ~30
// scalar / LDS instructions between chains).  One workgroup, one wave per SIMD; each mode issues 8 MFMAs on 8
// independent accumulators per iteration with the named filler after each MFMA (or after the group of 8).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_interleave.hip -o tools/mfma_interleave
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
#define M(i) "v_mfma_f64_16x16x4_f64 %[a" #i "], %[x], %[y], %[a" #i "]\n\t"
#define OPS [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]), [a4] "+v"(acc[4]), \
            [a5] "+v"(acc[5]), [a6] "+v"(acc[6]), [a7] "+v"(acc[7]), [s] "+s"(sc), [v] "+v"(vv), [l] "+v"(lv)
#define INS [x] "v"(x), [y] "v"(y), [addr] "v"(addr)
template <int MODE>
__global__ void k(double* out, unsigned long long* cyc, int iters) {
  __shared__ double lds[2048];
  f64x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f64x4{0, 0, 0, 0};
  double x = threadIdx.x * 1e-3, y = 1.0 + threadIdx.x * 1e-4;
  int sc = 1, vv = threadIdx.x;
  double lv = 0.0;
  const unsigned addr = (threadIdx.x & 63) * 8;
  lds[threadIdx.x] = x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0)   // straight chain
      asm volatile(M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) : OPS : INS);
    else if constexpr (MODE == 1)   // one SALU op after each MFMA
#define F "s_add_u32 %[s], %[s], 1\n\t"
      asm volatile(M(0) F M(1) F M(2) F M(3) F M(4) F M(5) F M(6) F M(7) F : OPS : INS : "scc");
#undef F
    else if constexpr (MODE == 2)   // one VALU op after each MFMA
#define F "v_add_u32 %[v], %[v], 1\n\t"
      asm volatile(M(0) F M(1) F M(2) F M(3) F M(4) F M(5) F M(6) F M(7) F : OPS : INS);
#undef F
    else if constexpr (MODE == 3)   // one LDS read after each MFMA
#define F "ds_read_b64 %[l], %[addr]\n\t"
      asm volatile(M(0) F M(1) F M(2) F M(3) F M(4) F M(5) F M(6) F M(7) F "s_waitcnt lgkmcnt(0)\n\t" : OPS : INS);
#undef F
    else if constexpr (MODE == 4)   // 24 SALU ops after the group of 8
#define F "s_add_u32 %[s], %[s], 1\n\t"
      asm volatile(M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) F F F F F F F F F F F F F F F F F F F F F F F F : OPS : INS : "scc");
#undef F
    else if constexpr (MODE == 5)   // an s_getpc / s_setpc jump after the group of 8
      asm volatile(M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
                   "s_getpc_b64 s[94:95]\n\ts_add_u32 s94, s94, 12\n\ts_addc_u32 s95, s95, 0\n\ts_setpc_b64 s[94:95]\n\t"
                   : OPS : INS : "scc", "s94", "s95");
    else if constexpr (MODE == 6)   // s_nop 1 before each MFMA (the old mfma_acc)
#define F "s_nop 1\n\t"
      asm volatile(F M(0) F M(1) F M(2) F M(3) F M(4) F M(5) F M(6) F M(7) : OPS : INS);
#undef F
    else if constexpr (MODE == 7)   // 6 LDS reads (b64) after the group of 8, waited for at the end
#define F "ds_read_b64 %[l], %[addr]\n\t"
      asm volatile(M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) F F F F F F "s_waitcnt lgkmcnt(0)\n\t" : OPS : INS);
#undef F
    else if constexpr (MODE == 8)   // 4 MFMAs then 12 SALU (a short chain per point)
#define F "s_add_u32 %[s], %[s], 1\n\t"
      asm volatile(M(0) M(1) M(2) M(3) F F F F F F F F F F F F M(4) M(5) M(6) M(7) F F F F F F F F F F F F : OPS : INS : "scc");
#undef F
    else if constexpr (MODE == 9) {   // v_mfma_f64_4x4x4_4b_f64 (4 blocks of 4x4x4) on 8 independent accumulators
      double d[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = acc[i][0];
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, d[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i][0] = d[i];
    }
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = lv + sc + vv;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
template <int MODE>
void run(double* out, unsigned long long* cyc, const char* name) {
  const int iters = 2000;
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k<MODE>, dim3(1), dim3(256), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("mode %d %-40s %.1f cycles per MFMA\n", MODE, name, (double)c / (iters * 8.0));
}
int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 1 << 16);
  hipMalloc(&cyc, 64);
  run<0>(out, cyc, "straight");
  run<1>(out, cyc, "1 SALU after each");
  run<2>(out, cyc, "1 VALU after each");
  run<3>(out, cyc, "1 ds_read_b64 after each");
  run<4>(out, cyc, "24 SALU after 8");
  run<5>(out, cyc, "getpc/setpc jump after 8");
  run<6>(out, cyc, "s_nop 1 before each");
  run<7>(out, cyc, "6 ds_read_b64 after 8");
  run<8>(out, cyc, "12 SALU after 4");
  run<9>(out, cyc, "v_mfma_f64_4x4x4_4b_f64 straight");
  return 0;
}
