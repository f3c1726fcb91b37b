// hamming.hip — all-pairs 256-bit descriptor matching (BASELINE config 4, the brute-force descriptor
// distance of the north star).  distance = popcount(a XOR b) over 4 x u64; per query
// the argmin over the train set (ties -> lowest train index) and the second-smallest distance.
//
// Matrix-core formulation.  With every bit expanded to an int8 of +-1 (query: bit -> +1 / -1, train: the
// opposite sign), the 256-term dot product is  dot(q', t') = -(256 - 2 h) = 2 h - 256  for Hamming distance h,
// so one v_mfma_i32_16x16x64_i8 chain of four K-steps with the accumulator starting at 256 leaves 2 h in every
// element of a 16 x 16 (query x train) tile: exact integer arithmetic, no popcount.  k_hamming_slices is a GEMM
// with the +-1 expansion fused into its loads (16 bits -> 16 bytes: a multiply-spread and v_bfi per nibble)
// and a fused arg-min epilogue:
//   * workgroup: 256 queries (8 waves = 4 query groups of 64 x 2 train halves of 64) against one slice of
//     the train set, streamed through LDS in tiles of 128 descriptors (272-byte rows: conflict-free
//     ds_read_b128), the next tile prefetched into registers during the current one;
//   * each wave keeps its 64 queries' A fragments in VGPRs for the whole slice (4 row tiles x 4 K-steps);
//   * epilogue per output: key = (2h << 22) | slice index (v_lshl_or), best = v_min, second = v_med3 — the
//     same packed-key rule as the VALU kernel (ties -> lowest index; second = the multiset's second key);
//   * per slice: a 16-lane butterfly merges each query's keys over the tile columns, LDS merges the two
//     train halves, one (best, index, second) triple per query and slice; k_hamming_merge combines slices
//     in slice order.
// The VALU popcount kernel this replaces (scalar-load train operands, 19 ops per pair) ran 70 us at
// 10k x 10k and was bound by v_bcnt issue.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <memory>
#include <vector>

#include "common.h"
#include "dbuf.h"

namespace sg {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));   // 16 int8 (one MFMA A/B fragment) or 4 int32 (C/D)

constexpr int kHmThreads = 512;              // 8 waves: 4 query groups x 2 train halves
constexpr int kHmQ = 256;                    // queries per workgroup
constexpr int kHmTile = 128;                 // train descriptors per LDS tile
constexpr int kHmPitch = 272;                // LDS bytes per descriptor row (256 + 16)
constexpr int kKeyShift = 22;                // slice index bits of the packed key (slices <= 2^22)
constexpr unsigned kKeyInf = 0xFFFFFFFFu;

// 4 bits -> 4 bytes of +-1: spread bit i to byte i ((n * 0x204081) & 0x01010101, no carries: the shifted
// copies do not overlap), make each set byte 0xFF ((s << 8) - s), then pick +1 / -1 per byte with v_bfi.
// pos: the byte of a set bit (+1 for queries, -1 for the train side); the clear bits get the other sign.
__device__ __forceinline__ int expand4(unsigned nib, unsigned pos, unsigned negv) {
  const unsigned s = __umul24(nib, 0x204081u) & 0x01010101u;
  const unsigned m = (s << 8) - s;
  return (int)((m & pos) | (~m & negv));   // v_bfi_b32
}
// 16 bits -> one A/B fragment (16 int8)
__device__ __forceinline__ v4i expand16(unsigned b, unsigned pos, unsigned negv) {
  v4i w;
  w[0] = expand4(b & 15u, pos, negv);
  w[1] = expand4((b >> 4) & 15u, pos, negv);
  w[2] = expand4((b >> 8) & 15u, pos, negv);
  w[3] = expand4((b >> 12) & 15u, pos, negv);
  return w;
}

__device__ __forceinline__ unsigned umed3(unsigned a, unsigned b, unsigned c) {
  unsigned r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ void ham_take(unsigned key, unsigned& m1, unsigned& m2) {
  m2 = umed3(m1, key, m2);   // second smallest (m1 <= m2)
  m1 = min(m1, key);
}

__device__ __forceinline__ void ham_merge(unsigned& m1, unsigned& m2, unsigned o1, unsigned o2) {
  const unsigned n2 = min(max(m1, o1), min(m2, o2));
  m1 = min(m1, o1);
  m2 = n2;
}

// qb / tb: the descriptors' bits, 16 uint16 (256 bits) per descriptor; expanded to +-1 int8 on the way in
// (A fragments once per workgroup, B tiles into LDS).
template <bool kPartial>
__device__ __forceinline__ void ham_tile(const v4i (&a)[4][4], const unsigned char* tile, int wi, int li, int g,
                                         int tbase, int cnt, unsigned (&m1)[4][4], unsigned (&m2)[4][4]) {
  const v4i cinit = {256, 256, 256, 256};
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int row = 64 * wi + 16 * ct + li;
    v4i acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const v4i bf = *reinterpret_cast<const v4i*>(tile + row * kHmPitch + 64 * k + 16 * g);
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
        acc[rt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[rt][k], bf, k == 0 ? cinit : acc[rt], 0, 0, 0);
    }
    // acc[rt][r] = 2 h of query 16 rt + 4 g + r and train descriptor tbase + row (slice index)
    const unsigned idx = (unsigned)(tbase + row);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        unsigned key = ((unsigned)acc[rt][r] << kKeyShift) | idx;
        if (kPartial) key = (int)idx < cnt ? key : kKeyInf;
        ham_take(key, m1[rt][r], m2[rt][r]);
      }
  }
}

__global__ __launch_bounds__(kHmThreads) void k_hamming_slices(const uint16_t* __restrict__ qb, int nq,
                                                               const uint16_t* __restrict__ tb, int nt, int slice_len,
                                                               int3* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) unsigned char tile[kHmTile * kHmPitch];
  __shared__ unsigned red[4][64][2];
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wq = wave & 3, wi = wave >> 2;
  const int s = blockIdx.y;
  const int j0 = min(nt, s * slice_len), cnt = min(slice_len, nt - j0);
  const int qbase = blockIdx.x * kHmQ + 64 * wq;
  // A fragments: row tile rt, K-step k: query qbase + 16 rt + li, bytes 64 k + 16 g
  v4i a[4][4];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) {
    const int qi = min(qbase + 16 * rt + li, nq - 1);   // nq >= 1 (nothing is launched for nq == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) a[rt][k] = expand16(qb[(size_t)qi * 16 + 4 * k + g], 0x01010101u, 0xFFFFFFFFu);
  }
  unsigned m1[4][4], m2[4][4];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) m1[rt][r] = m2[rt][r] = kKeyInf;
  const int ntile = (cnt + kHmTile - 1) / kHmTile;
  // tile loads: 128 descriptors x 16 chunks of 16 bits, 4 chunks per thread (chunk c: descriptor c >> 4,
  // bits 16 (c & 15) ..); descriptors past the slice end read the slice's last one (masked in the epilogue);
  // each chunk is expanded to a 16-byte fragment (train side: set bit -> -1) on its way into LDS
  unsigned pre[4];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + kHmThreads * u;
      const int item = min(t * kHmTile + (c >> 4), cnt - 1);
      pre[u] = tb[(size_t)(j0 + item) * 16 + (c & 15)];
    }
  };
  if (ntile > 0) load_tile(0);
  for (int t = 0; t < ntile; ++t) {
    __syncthreads();   // the previous tile's fragments are read
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + kHmThreads * u;
      *reinterpret_cast<v4i*>(tile + (c >> 4) * kHmPitch + 16 * (c & 15)) = expand16(pre[u], 0xFFFFFFFFu, 0x01010101u);
    }
    __syncthreads();
    if (t + 1 < ntile) load_tile(t + 1);
    if ((t + 1) * kHmTile > cnt)
      ham_tile<true>(a, tile, wi, li, g, t * kHmTile, cnt, m1, m2);
    else
      ham_tile<false>(a, tile, wi, li, g, t * kHmTile, cnt, m1, m2);
  }
  // merge over the 16 tile columns (lanes of a 16-lane group)
#pragma unroll
  for (int mask = 1; mask < 16; mask <<= 1)
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const unsigned o1 = __shfl_xor(m1[rt][r], mask), o2 = __shfl_xor(m2[rt][r], mask);
        ham_merge(m1[rt][r], m2[rt][r], o1, o2);
      }
  // lane li of group g takes query 16 (li >> 2) + 4 g + (li & 3) of the wave's 64
  unsigned k1 = kKeyInf, k2 = kKeyInf;
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (li == 4 * rt + r) {
        k1 = m1[rt][r];
        k2 = m2[rt][r];
      }
  const int ql = 16 * (li >> 2) + 4 * g + (li & 3);
  if (wi == 1) {
    red[wq][ql][0] = k1;
    red[wq][ql][1] = k2;
  }
  __syncthreads();
  if (wi == 1) return;
  ham_merge(k1, k2, red[wq][ql][0], red[wq][ql][1]);
  const int q = qbase + ql;
  if (q >= nq) return;
  const int bd = k1 == kKeyInf ? (1 << 30) : (int)(k1 >> (kKeyShift + 1));
  const int bi = k1 == kKeyInf ? -1 : j0 + (int)(k1 & ((1u << kKeyShift) - 1));
  const int sd = k2 == kKeyInf ? (1 << 30) : (int)(k2 >> (kKeyShift + 1));
  part[(size_t)s * nq + q] = make_int3(bd, bi, sd);
}

__global__ void k_hamming_merge(const int3* __restrict__ part, int nq, int nslice, int nt, int32_t* best_idx,
                                int32_t* best_dist, int32_t* second_dist) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  int bd = 1 << 30, bi = -1, sd = 1 << 30;
  for (int s0 = 0; s0 < nslice; s0 += 8) {   // slice order = train index order; 8 partials in flight
    int3 p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] = part[(size_t)min(s0 + u, nslice - 1) * nq + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (s0 + u >= nslice) break;
      if (p[u].x < bd) {
        sd = min(bd, p[u].z);
        bd = p[u].x;
        bi = p[u].y;
      } else {
        sd = min(sd, p[u].x);
      }
    }
  }
  best_idx[i] = bi;
  best_dist[i] = nt > 0 ? bd : -1;
  second_dist[i] = nt > 1 ? sd : -1;
}

}  // namespace

class HammingMatcher {
 public:
  explicit HammingMatcher(const sg_device_options& d) : dev_(d) {
    int ndev = 0;
    SG_HIP_CHECK(hipGetDeviceCount(&ndev));
    SG_REQUIRE(ndev > 0 && d.device >= 0 && d.device < ndev, SG_ENODEV, "no such HIP device");
    SG_HIP_CHECK(hipSetDevice(d.device));
    SG_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    SG_HIP_CHECK(hipEventCreate(&e0_));
    SG_HIP_CHECK(hipEventCreate(&e1_));
  }
  ~HammingMatcher() {
    (void)hipSetDevice(dev_.device);
    if (e0_) (void)hipEventDestroy(e0_);
    if (e1_) (void)hipEventDestroy(e1_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }

  void Load(const uint64_t* q, int nq, const uint64_t* t, int nt) {
    SG_REQUIRE(nq >= 0 && nt >= 0 && (nq == 0 || q) && (nt == 0 || t), SG_EINVAL, "bad descriptors");
    SG_HIP_CHECK(hipSetDevice(dev_.device));
    nq_ = nq;
    nt_ = nt;
    q_.Upload(std::vector<uint64_t>(q, q + 4 * (size_t)nq), stream_);
    t_.Upload(std::vector<uint64_t>(t, t + 4 * (size_t)nt), stream_);
    // about two rounds of one workgroup per CU (214 VGPRs: one 8-wave workgroup fits a CU; measured better
    // than one longer round); slices are whole 128-descriptor tiles except the last, < 2^22
    const int qg = std::max(1, (nq + kHmQ - 1) / kHmQ);
    nslice_ = std::max(1, std::min((512 + qg - 1) / qg, (nt + kHmTile - 1) / kHmTile));
    nslice_ = std::max(nslice_, (int)(((int64_t)nt + ((int64_t)1 << 21) - 1) >> 21));
    slice_len_ = std::max(kHmTile, ((nt + nslice_ - 1) / nslice_ + kHmTile - 1) / kHmTile * kHmTile);
    nslice_ = std::max(1, (nt + slice_len_ - 1) / slice_len_);
    part_.Resize((size_t)nslice_ * std::max(nq, 1) * 3);
    bi_.Resize(std::max(nq, 1));
    bd_.Resize(std::max(nq, 1));
    sd_.Resize(std::max(nq, 1));
  }

  void Run(int repeats) {
    SG_REQUIRE(repeats >= 1, SG_EINVAL, "repeats must be >= 1");
    SG_HIP_CHECK(hipSetDevice(dev_.device));
    SG_HIP_CHECK(hipEventRecord(e0_, stream_));
    if (nq_ > 0)
      for (int r = 0; r < repeats; ++r) {
        hipLaunchKernelGGL(k_hamming_slices, dim3((nq_ + kHmQ - 1) / kHmQ, nslice_), dim3(kHmThreads), 0, stream_,
                           (const uint16_t*)q_.ptr, nq_, (const uint16_t*)t_.ptr, nt_, slice_len_, (int3*)part_.ptr);
        hipLaunchKernelGGL(k_hamming_merge, dim3((nq_ + 255) / 256), dim3(256), 0, stream_, (const int3*)part_.ptr,
                           nq_, nslice_, nt_, bi_.ptr, bd_.ptr, sd_.ptr);
      }
    SG_HIP_CHECK(hipEventRecord(e1_, stream_));
    SG_HIP_CHECK(hipGetLastError());
    ran_ = true;
    repeats_ = repeats;
  }

  void Results(int32_t* bi, int32_t* bd, int32_t* sd, double* ms) {
    SG_REQUIRE(ran_, SG_EINVAL, "no matching run");
    SG_HIP_CHECK(hipSetDevice(dev_.device));
    if (nq_ > 0) {
      if (bi) SG_HIP_CHECK(hipMemcpyAsync(bi, bi_.ptr, 4 * (size_t)nq_, hipMemcpyDeviceToHost, stream_));
      if (bd) SG_HIP_CHECK(hipMemcpyAsync(bd, bd_.ptr, 4 * (size_t)nq_, hipMemcpyDeviceToHost, stream_));
      if (sd) SG_HIP_CHECK(hipMemcpyAsync(sd, sd_.ptr, 4 * (size_t)nq_, hipMemcpyDeviceToHost, stream_));
    }
    SG_HIP_CHECK(hipStreamSynchronize(stream_));
    float t = 0.f;
    SG_HIP_CHECK(hipEventElapsedTime(&t, e0_, e1_));
    if (ms) *ms = t / repeats_;
  }

 private:
  sg_device_options dev_;
  hipStream_t stream_ = nullptr;
  hipEvent_t e0_ = nullptr, e1_ = nullptr;
  DBuf<uint64_t> q_, t_;
  DBuf<int32_t> part_, bi_, bd_, sd_;
  int nq_ = 0, nt_ = 0, nslice_ = 1, slice_len_ = 1, repeats_ = 1;
  bool ran_ = false;
};

}  // namespace sg

struct sg_matcher {
  std::unique_ptr<sg::HammingMatcher> m;
};

extern "C" {

int sg_matcher_create(sg_matcher** out, const sg_device_options* dev) {
  SG_CAPI_BEGIN
  SG_REQUIRE(out, SG_EINVAL, "null output handle");
  sg_device_options d;
  sg_device_options_default(&d);
  if (dev) d = *dev;
  auto h = std::make_unique<sg_matcher>();
  h->m.reset(new sg::HammingMatcher(d));
  *out = h.release();
  SG_CAPI_END
}

void sg_matcher_destroy(sg_matcher* m) { delete m; }

int sg_hamming_load(sg_matcher* m, const uint64_t* query, int32_t nq, const uint64_t* train, int32_t nt) {
  SG_CAPI_BEGIN
  SG_REQUIRE(m, SG_EINVAL, "null handle");
  m->m->Load(query, nq, train, nt);
  SG_CAPI_END
}

int sg_hamming_run(sg_matcher* m, int32_t repeats) {
  SG_CAPI_BEGIN
  SG_REQUIRE(m, SG_EINVAL, "null handle");
  m->m->Run(repeats);
  SG_CAPI_END
}

int sg_hamming_results(sg_matcher* m, int32_t* best_idx, int32_t* best_dist, int32_t* second_dist, double* kernel_ms) {
  SG_CAPI_BEGIN
  SG_REQUIRE(m, SG_EINVAL, "null handle");
  m->m->Results(best_idx, best_dist, second_dist, kernel_ms);
  SG_CAPI_END
}

int sg_hamming_match(sg_matcher* m, const uint64_t* query, int32_t nq, const uint64_t* train, int32_t nt,
                     int32_t* best_idx, int32_t* best_dist, int32_t* second_dist) {
  SG_CAPI_BEGIN
  SG_REQUIRE(m && (nq == 0 || (best_idx && best_dist && second_dist)), SG_EINVAL, "null argument");
  m->m->Load(query, nq, train, nt);
  m->m->Run(1);
  m->m->Results(best_idx, best_dist, second_dist, nullptr);
  SG_CAPI_END
}

}  // extern "C"
