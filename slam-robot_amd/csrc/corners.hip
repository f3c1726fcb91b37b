// corners.hip — corner seeding of a new keyframe on the device: Matcher::Track's
// cvtColor(img, grey, CV_RGB2GRAY) (matcher.cpp:214), goodFeaturesToTrack(grey, corners, 120, 0.01, 20)
// (matcher.cpp:125-130, OpenCV 2.4 defaults: blockSize 3, Shi-Tomasi minimum eigenvalue) and
// AddNewFeatures' 30 x 30 grid suppression around the current matches (matcher.cpp:132-168).
//
//   k_grey_u8     BGR u8 -> grey u8 (the RGB2GRAY weights on BGR memory, fixed point), kept per slot
//   k_sobel       Sobel 3x3 dx, dy scaled by 1 / (4 * 3 * 255) on the smoothing tap (BORDER_REFLECT_101)
//   k_min_eigen   3x3 unnormalised box sums of (dx^2, dx dy, dy^2), lambda_min, block max -> atomicMax
//   k_candidates  THRESH_TOZERO at quality x max, 3x3 local maxima (the dilate == value test)
//   hipCUB        order-preserving compaction of the candidates, stable radix sort by response
//                 (descending; equal responses keep row-major order)
//   k_select      one wave: greedy minimum-distance acceptance in response order (batches of 64
//                 candidates tested against the accepted set in parallel, resolved in order by ballots),
//                 then the grid filter against the matches
// Float arithmetic follows the oracle (oracle_track.cpp MinEigen3 / GoodFeatures) operation for operation
// with contraction off, so responses, candidates and corners are bit-identical to the oracle's.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "tracker.h"

#pragma clang fp contract(off)

namespace sg {

namespace {

__device__ __forceinline__ int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
  }
  return p;
}

}  // namespace

__global__ void k_grey_u8(const uint8_t* bgr, int w, int h, int stride, uint8_t* grey) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const uint8_t* p = bgr + (size_t)y * stride + 3 * x;
  grey[(size_t)y * w + x] = (uint8_t)((4899 * p[0] + 9617 * p[1] + 1868 * p[2] + (1 << 13)) >> 14);
}

namespace {

constexpr int kSelThreads = 64;
constexpr int kMaxSeed = 1024;   // accepted corners held in LDS

__global__ void k_sobel(const uint8_t* g, int w, int h, float* dx, float* dy) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const float s = (float)(1.0 / (4.0 * 3.0 * 255.0));
  const float k0 = 2.0f * s, k1 = s;
  const int xm = reflect101(x - 1, w), xp = reflect101(x + 1, w);
  float r[3], q[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const uint8_t* row = g + (size_t)reflect101(y - 1 + k, h) * w;
    const float a = row[xm], b = row[x], c = row[xp];
    r[k] = c - a;
    q[k] = b * k0 + (a + c) * k1;
  }
  dx[(size_t)y * w + x] = r[1] * k0 + (r[0] + r[2]) * k1;
  dy[(size_t)y * w + x] = q[2] - q[0];
}

__global__ __launch_bounds__(256) void k_min_eigen(const float* dx, const float* dy, int w, int h, float* eig,
                                                   unsigned int* maxbits) {
  __shared__ float red[4];
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  float v = 0.0f;
  if (x < w) {
    const int xs[3] = {reflect101(x - 1, w), x, reflect101(x + 1, w)};
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const size_t row = (size_t)reflect101(y - 1 + k, h) * w;
      float c0[3], c1[3], c2[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float a = dx[row + xs[j]], b = dy[row + xs[j]];
        c0[j] = a * a;
        c1[j] = a * b;
        c2[j] = b * b;
      }
      const float r0 = (c0[0] + c0[1]) + c0[2], r1 = (c1[0] + c1[1]) + c1[2], r2 = (c2[0] + c2[1]) + c2[2];
      if (k == 0) {
        s0 = r0;
        s1 = r1;
        s2 = r2;
      } else {
        s0 = s0 + r0;
        s1 = s1 + r1;
        s2 = s2 + r2;
      }
    }
    const float a = s0 * 0.5f, b = s1, c = s2 * 0.5f;
    v = (a + c) - sqrtf((a - c) * (a - c) + b * b);
    eig[(size_t)y * w + x] = v;
  }
  // workgroup max of the non-negative part (float bit patterns of non-negative values order like them)
  float m = fmaxf(v, 0.0f);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = red[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) b = fmaxf(b, red[i]);
    atomicMax(maxbits, __float_as_uint(b));
  }
}

__global__ void k_candidates(const float* eig, int w, int h, const unsigned int* maxbits, double quality,
                             uint8_t* flag, float* val) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const size_t i = (size_t)y * w + x;
  const float thr = (float)((double)__uint_as_float(*maxbits) * quality);
  uint8_t f = 0;
  float v = 0.0f;
  if (x >= 1 && x < w - 1 && y >= 1 && y < h - 1) {
    v = eig[i];
    v = v > thr ? v : 0.0f;
    float m = v;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const float u = eig[i + (ptrdiff_t)dy * w + dx];
        m = fmaxf(m, u > thr ? u : 0.0f);
      }
    f = (v != 0.0f && v == m) ? 1 : 0;
  }
  flag[i] = f;
  val[i] = v;
}

// AddNewFeatures' cell of a point: (pt / size) * 30 + 1 in float, truncated (matcher.cpp:135-137).
__device__ __forceinline__ int seed_cell(float v, int size) { return (int)(v / size * 30 + 1); }

// One wave.  Candidates sorted by response (descending, ties in row-major order).
__global__ __launch_bounds__(kSelThreads) void k_select(const int* idx, int ncand, int w, int h, int max_corners,
                                                        float min_d2, const float* match_xy, int nmatch,
                                                        float* corners, int* counts, float* added) {
  __shared__ float ax[kMaxSeed], ay[kMaxSeed];
  __shared__ int grid[32 * 32];
  const int lane = threadIdx.x;
  int n = 0;   // wave-uniform
  for (int base = 0; base < ncand && n < max_corners; base += kSelThreads) {
    const int c = base + lane;
    const bool in = c < ncand;
    const int pi = in ? idx[c] : 0;
    const float x = (float)(pi % w), y = (float)(pi / w);
    bool good = in;
    for (int j = 0; j < n && good; ++j) {
      const float ddx = x - ax[j], ddy = y - ay[j];
      if (ddx * ddx + ddy * ddy < min_d2) good = false;
    }
    // resolve the batch in candidate order: the first still-good lane is accepted, the rest test against it
    unsigned long long alive = __ballot(good);
    while (alive && n < max_corners) {
      const int l = __ffsll(alive) - 1;
      const float bx = __shfl(x, l), by = __shfl(y, l);
      if (lane == 0) {
        ax[n] = bx;
        ay[n] = by;
      }
      ++n;
      if (lane > l && good) {
        const float ddx = x - bx, ddy = y - by;
        if (ddx * ddx + ddy * ddy < min_d2) good = false;
      }
      if (lane == l) good = false;
      alive = __ballot(good);
    }
    __syncthreads();
  }
  // AddNewFeatures: cells around the matches, then the corners in order
  for (int i = lane; i < 32 * 32; i += kSelThreads) grid[i] = 0;
  __syncthreads();
  for (int i = lane; i < nmatch; i += kSelThreads) {
    const int gx = seed_cell(match_xy[2 * i], w), gy = seed_cell(match_xy[2 * i + 1], h);
    if (gx <= 0 || gy <= 0 || gx >= 31 || gy >= 31) {
      atomicOr(counts + 2, 1);   // the reference CHECK-fails on such a match
      continue;
    }
    for (int a = -1; a <= 1; ++a)
      for (int b = -1; b <= 1; ++b) grid[(gx + a) * 32 + gy + b] = 1;
  }
  __syncthreads();
  int nadd = 0;
  for (int base = 0; base < n; base += kSelThreads) {
    const int i = base + lane;
    bool keep = false;
    float x = 0.0f, y = 0.0f;
    if (i < n) {
      x = ax[i];
      y = ay[i];
      corners[2 * i] = x;
      corners[2 * i + 1] = y;
      keep = grid[seed_cell(x, w) * 32 + seed_cell(y, h)] == 0;
    }
    const unsigned long long kb = __ballot(keep);
    if (keep) {
      const int pos = nadd + __popcll(kb & ((1ull << lane) - 1ull));
      added[2 * pos] = x;
      added[2 * pos + 1] = y;
    }
    nadd += __popcll(kb);
  }
  if (lane == 0) {
    counts[0] = n;
    counts[1] = nadd;
  }
}

}  // namespace

// goodFeaturesToTrack + AddNewFeatures on the grey image of `slot`.
void Tracker::SeedFeatures(int slot, const float* match_xy, int nmatch, int max_corners, double quality,
                           double min_distance, float* corners_xy, int* ncorners, float* added_xy, int* nadded) {
  SG_REQUIRE(slot >= 0 && slot < (int)slots_.size() && slots_[slot].valid, SG_EINVAL, "empty slot");
  SG_REQUIRE(max_corners >= 1 && max_corners <= kMaxSeed, SG_EINVAL, "max_corners must be 1..1024");
  SG_REQUIRE(min_distance >= 1.0 && quality > 0.0, SG_EINVAL, "min_distance must be >= 1, quality > 0");
  SG_REQUIRE(nmatch >= 0 && (nmatch == 0 || match_xy), SG_EINVAL, "bad matches");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  Slot& s = slots_[slot];
  const int w = s.w[0], h = s.h[0];
  const size_t np = (size_t)w * h;
  hipStream_t st = stream_;
  seed_dx_.Resize(np);
  seed_dy_.Resize(np);
  seed_eig_.Resize(np);
  seed_val_.Resize(np);
  seed_flag_.Resize(np);
  seed_idx_.Resize(np + 1);
  seed_val2_.Resize(np);
  seed_idx2_.Resize(np);
  seed_misc_.Resize(4);
  seed_misc_.Zero(st);
  const int bx = 256;
  const dim3 grid2((w + bx - 1) / bx, h);
  hipLaunchKernelGGL(k_sobel, grid2, dim3(bx), 0, st, s.grey.ptr, w, h, seed_dx_.ptr, seed_dy_.ptr);
  hipLaunchKernelGGL(k_min_eigen, grid2, dim3(bx), 0, st, seed_dx_.ptr, seed_dy_.ptr, w, h, seed_eig_.ptr,
                     reinterpret_cast<unsigned int*>(seed_misc_.ptr));
  hipLaunchKernelGGL(k_candidates, grid2, dim3(bx), 0, st, seed_eig_.ptr, w, h,
                     reinterpret_cast<const unsigned int*>(seed_misc_.ptr), quality, seed_flag_.ptr, seed_val_.ptr);
  SG_HIP_CHECK(hipGetLastError());
  // compaction in pixel order, then a stable descending sort by response
  int* d_num = seed_misc_.ptr + 1;
  hipcub::CountingInputIterator<int> counting(0);
  size_t tb_sel = 0, tb_sort = 0;
  SG_HIP_CHECK(hipcub::DeviceSelect::Flagged(nullptr, tb_sel, counting, seed_flag_.ptr, seed_idx_.ptr, d_num,
                                             (int)np, st));
  SG_HIP_CHECK(hipcub::DeviceSelect::Flagged(nullptr, tb_sel, seed_val_.ptr, seed_flag_.ptr, seed_val2_.ptr, d_num,
                                             (int)np, st));
  SG_HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb_sort, seed_val2_.ptr, seed_eig_.ptr,
                                                            seed_idx_.ptr, seed_idx2_.ptr, (int)np, 0, 32, st));
  seed_tmp_.Resize(std::max(std::max(tb_sel, tb_sort), (size_t)1));
  SG_HIP_CHECK(hipcub::DeviceSelect::Flagged(seed_tmp_.ptr, tb_sel, counting, seed_flag_.ptr, seed_idx_.ptr, d_num,
                                             (int)np, st));
  int ncand = 0;
  SG_HIP_CHECK(hipMemcpyAsync(&ncand, d_num, sizeof(int), hipMemcpyDeviceToHost, st));
  SG_HIP_CHECK(hipcub::DeviceSelect::Flagged(seed_tmp_.ptr, tb_sel, seed_val_.ptr, seed_flag_.ptr, seed_val2_.ptr,
                                             d_num, (int)np, st));
  SG_HIP_CHECK(hipStreamSynchronize(st));
  if (ncand > 0) {
    // keys: the candidates' responses (in pixel order); the sorted keys land in the (free) eig buffer
    SG_HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(seed_tmp_.ptr, tb_sort, seed_val2_.ptr, seed_eig_.ptr,
                                                              seed_idx_.ptr, seed_idx2_.ptr, ncand, 0, 32, st));
  }
  DBuf<float> dm, dc, da;
  dm.Upload(nmatch ? std::vector<float>(match_xy, match_xy + 2 * (size_t)nmatch) : std::vector<float>(2, 0.f), st);
  dc.Resize(2 * (size_t)max_corners);
  da.Resize(2 * (size_t)max_corners);
  const float md2 = (float)(min_distance * min_distance);
  hipLaunchKernelGGL(k_select, dim3(1), dim3(kSelThreads), 0, st, seed_idx2_.ptr, ncand, w, h, max_corners, md2,
                     dm.ptr, nmatch, dc.ptr, seed_misc_.ptr + 1, da.ptr);
  SG_HIP_CHECK(hipGetLastError());
  int cnt[3] = {0, 0, 0};
  SG_HIP_CHECK(hipMemcpyAsync(cnt, seed_misc_.ptr + 1, 3 * sizeof(int), hipMemcpyDeviceToHost, st));
  SG_HIP_CHECK(hipStreamSynchronize(st));
  SG_REQUIRE(cnt[2] == 0, SG_EINVAL, "a match lies outside the image (AddNewFeatures CHECK)");
  *ncorners = cnt[0];
  *nadded = cnt[1];
  if (cnt[0]) SG_HIP_CHECK(hipMemcpyAsync(corners_xy, dc.ptr, 2 * sizeof(float) * cnt[0], hipMemcpyDeviceToHost, st));
  if (cnt[1]) SG_HIP_CHECK(hipMemcpyAsync(added_xy, da.ptr, 2 * sizeof(float) * cnt[1], hipMemcpyDeviceToHost, st));
  SG_HIP_CHECK(hipStreamSynchronize(st));
}

}  // namespace sg
