// tracker.hip — MI355X-native front end: the reference's HessianTracker (hessian.h) and the
// forward/backward matching step of Matcher (matcher.cpp:173-206, 247-251).
//
//   pyramid   MakePyramid (hessian.h:95-126): BGR u8 -> grey (CV_RGB2GRAY weights on channel 0) -> /255
//             -> GaussianBlur 5x5 sigma 1.1; per level pyrDown + GaussianBlur 5x5 sigma 0.8.  Stencil
//             kernels, one thread per output pixel, BORDER_REFLECT_101.
//   tracking  one wavefront per feature.  Lane l owns patch pixels l, l+64, ... ; the six Newton probes of
//             BruteHessian (hessian.h:147-172) are sampled together, their mean / sumsq / score sums are
//             reduced by DPP wave reductions in a batch, and the 2x2 Newton step of Track (185-241) runs
//             in fp64 as in the reference.  TrackFeature (243-264) walks the levels coarse to fine; the
//             matcher's forward pass, backward pass, 0.3 px check and 3 -> 6 level retry all run in the
//             same wave.
//
// Arithmetic follows the oracle (oracle/oracle_track.cpp) operation for operation with FMA contraction
// off, and the patch sums use the oracle's fixed order (64 lane-strided partials + pairwise tree), so the
// device results are bit-identical to the oracle's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.h"
#include "tracker.h"

#pragma clang fp contract(off)

namespace sg {

namespace {

constexpr int kTrackWaves = 4;   // features per workgroup (one wave each)
constexpr int kNP = 4;           // patch pixels per lane (W <= 16)

__device__ __forceinline__ int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
  }
  return p;
}

// ------------------------------------------------------------------------------------------------
// Pyramid kernels

struct Blur5 {
  float k0, k1, k2;
};

// level 0, row pass: grey u8 (computed from BGR on the fly) -> float /255 -> 5-tap row blur
__global__ void k_gray_blur_row(const uint8_t* bgr, int w, int h, int stride, Blur5 k, float* out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  const uint8_t* row = bgr + (size_t)y * stride;
  const float sc = (float)(1. / 255.);
  auto g = [&](int xx) {
    const uint8_t* p = row + 3 * reflect101(xx, w);
    const int v = (4899 * p[0] + 9617 * p[1] + 1868 * p[2] + (1 << 13)) >> 14;
    return (float)(uint8_t)v * sc;
  };
  const float c = g(x), l1 = g(x - 1), r1 = g(x + 1), l2 = g(x - 2), r2 = g(x + 2);
  out[(size_t)y * w + x] = c * k.k0 + (l1 + r1) * k.k1 + (l2 + r2) * k.k2;
}

// level 0 of the klt.h / brute.h pyramids (klt.h:104, brute.h:64): grey / 255, no blur
__global__ void k_gray_scale(const uint8_t* bgr, int w, int h, int stride, float* out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  const uint8_t* p = bgr + (size_t)y * stride + 3 * x;
  const int v = (4899 * p[0] + 9617 * p[1] + 1868 * p[2] + (1 << 13)) >> 14;
  out[(size_t)y * w + x] = (float)(uint8_t)v * (float)(1. / 255.);
}

__global__ void k_blur_row(const float* in, int w, int h, Blur5 k, float* out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  const float* r = in + (size_t)y * w;
  const float c = r[x], l1 = r[reflect101(x - 1, w)], r1 = r[reflect101(x + 1, w)];
  const float l2 = r[reflect101(x - 2, w)], r2 = r[reflect101(x + 2, w)];
  out[(size_t)y * w + x] = c * k.k0 + (l1 + r1) * k.k1 + (l2 + r2) * k.k2;
}

__global__ void k_blur_col(const float* in, int w, int h, Blur5 k, float* out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  const float c = in[(size_t)y * w + x];
  const float u1 = in[(size_t)reflect101(y - 1, h) * w + x], d1 = in[(size_t)reflect101(y + 1, h) * w + x];
  const float u2 = in[(size_t)reflect101(y - 2, h) * w + x], d2 = in[(size_t)reflect101(y + 2, h) * w + x];
  out[(size_t)y * w + x] = c * k.k0 + (u1 + d1) * k.k1 + (u2 + d2) * k.k2;
}

// pyrDown: the row pass values of the five source rows are recomputed per output (same arithmetic as the
// separable form), then combined 1-4-6-4-1 and scaled by 1/256.
__global__ void k_pyrdown(const float* in, int w, int h, float* out, int ow, int oh) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= ow || y >= oh) return;
  const int c = 2 * x;
  const int cm2 = reflect101(c - 2, w), cm1 = reflect101(c - 1, w), c0 = reflect101(c, w);
  const int cp1 = reflect101(c + 1, w), cp2 = reflect101(c + 2, w);
  float rv[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const float* s = in + (size_t)reflect101(2 * y + k - 2, h) * w;
    rv[k] = s[c0] * 6 + (s[cm1] + s[cp1]) * 4 + s[cm2] + s[cp2];
  }
  out[(size_t)y * ow + x] = (rv[2] * 6 + (rv[1] + rv[3]) * 4 + rv[0] + rv[4]) * (1.f / 256.f);
}

// ------------------------------------------------------------------------------------------------
// Patch sampling (GetPatch = zero-filled left/top edge + getRectSubPix) and reductions

struct LevelDev {
  const float* img;
  int w, h;
};
struct PyrDev {
  LevelDev lv[kTrkMaxDepth];
  int depth;
};

// Per-probe geometry (wave-uniform).
struct Geo {
  int zx, zy;               // zero-filled columns / rows of the W x W patch (GetPatch, hessian.h:63-75)
  int pw, ph;               // getRectSubPix window (W - zx) x (W - zy)
  int col0, base_row;       // adjustRect: source column of window column 0 (minus rect.x), first row
  int rx, rw, ry, rh;       // adjustRect rect
  float a11, a12, a21, a22, b1, b2;
};

// make_geo's two halves: the column geometry depends on px alone, the row geometry on py alone (the Newton
// probes share them three ways, brute_hessian).
struct GeoX {
  int zx, pw, col0, rx, rw;
  float a;
};
struct GeoY {
  int zy, ph, base_row, ry, rh;
  float b;
};
// kShift: HessianTracker::GetPatch's zero-filled left / top edge (hessian.h:63-75); without it the plain
// getRectSubPix of klt.h / brute.h GetPatch.
template <bool kShift = true>
__device__ __forceinline__ void make_geo_x(float px, int W, int w, GeoX& g) {
  g.zx = 0;
  g.pw = W;
  if (kShift && px < 0.5 * W) {
    const int d = (int)((0.5 * W - px) + 0.9999);
    px = (float)(px + 0.5 * d);
    g.zx = d;
    g.pw = W - d;
  }
  const float cx = px - (g.pw - 1) * 0.5f;
  const int ipx = (int)floorf(cx);
  g.a = cx - ipx;
  int base_col;
  if (ipx >= 0) { base_col = ipx; g.rx = 0; }
  else { base_col = 0; g.rx = min(-ipx, g.pw); }
  if (ipx < w - g.pw) g.rw = g.pw;
  else {
    g.rw = w - ipx - 1;
    if (g.rw < 0) { base_col += g.rw; g.rw = 0; }
  }
  g.col0 = base_col - g.rx;
}
template <bool kShift = true>
__device__ __forceinline__ void make_geo_y(float py, int W, int h, GeoY& g) {
  g.zy = 0;
  g.ph = W;
  if (kShift && py < 0.5 * W) {
    const int d = (int)(0.5 * W - py);
    py = (float)(py + 0.5 * d);
    g.zy = d;
    g.ph = W - d;
  }
  const float cy = py - (g.ph - 1) * 0.5f;
  const int ipy = (int)floorf(cy);
  g.b = cy - ipy;
  if (ipy >= 0) { g.base_row = ipy; g.ry = 0; }
  else { g.base_row = 0; g.ry = -ipy; }
  if (ipy < h - g.ph) g.rh = g.ph;
  else {
    g.rh = h - ipy - 1;
    if (g.rh < 0) { g.base_row += g.rh; g.rh = 0; }
  }
}
__device__ __forceinline__ void geo_join(const GeoX& x, const GeoY& y, Geo& g) {
  g.zx = x.zx;
  g.pw = x.pw;
  g.col0 = x.col0;
  g.rx = x.rx;
  g.rw = x.rw;
  g.zy = y.zy;
  g.ph = y.ph;
  g.base_row = y.base_row;
  g.ry = y.ry;
  g.rh = y.rh;
  const float a = x.a, b = y.b;
  g.a11 = (1.f - a) * (1.f - b);
  g.a12 = a * (1.f - b);
  g.a21 = (1.f - a) * b;
  g.a22 = a * b;
  g.b1 = 1.f - b;
  g.b2 = b;
}
__device__ __forceinline__ bool geo_x_same(const GeoX& p, const GeoX& q) {
  return p.zx == q.zx && p.pw == q.pw && p.col0 == q.col0 && p.rx == q.rx && p.rw == q.rw;
}
__device__ __forceinline__ bool geo_y_same(const GeoY& p, const GeoY& q) {
  return p.zy == q.zy && p.ph == q.ph && p.base_row == q.base_row && p.ry == q.ry && p.rh == q.rh;
}
template <bool kShift = true>
__device__ __forceinline__ void make_geo(float px, float py, int W, int w, int h, Geo& g) {
  GeoX gx;
  GeoY gy;
  make_geo_x<kShift>(px, W, w, gx);
  make_geo_y<kShift>(py, W, h, gy);
  geo_join(gx, gy, g);
}

// Patch pixel (i, j) of the W x W patch: the four taps (taps) and their bilinear / edge combination (combine).
// Branch-free form of getRectSubPix's three cases (left edge column, interior bilinear, right edge column) and
// the zero-filled border: the four loads are unconditional (clamped to index 0 when the pixel is zero) so a
// wave's samples are all in flight together; each case's arithmetic is the reference expression, evaluated as
// written (FMA contraction is off in this file).
struct Taps {
  float v11, v12, v21, v22;
  bool zero, edge;
};
__device__ __forceinline__ float combine(const Taps& t, const Geo& g) {
  const float re = t.v11 * g.b1 + t.v21 * g.b2;
  const float rb = t.v11 * g.a11 + t.v12 * g.a12 + t.v21 * g.a21 + t.v22 * g.a22;
  return t.zero ? 0.f : (t.edge ? re : rb);
}
// combine() as selects only: both forms are formed (same expressions, so the same bits), then picked; `on` false
// (a slot past the patch) gives 0 as well.  (The ?: of combine() compiles to branches around the arithmetic.)
__device__ __forceinline__ float combine_sel(const Taps& t, const Geo& g, bool on) {
  float re = t.v11 * g.b1 + t.v21 * g.b2;
  float rb = t.v11 * g.a11 + t.v12 * g.a12 + t.v21 * g.a21 + t.v22 * g.a22;
  asm volatile("" : "+v"(re), "+v"(rb));
  const float r = t.edge ? re : rb;
  return (t.zero || !on) ? 0.f : r;
}
__device__ __forceinline__ Taps taps_global(const float* img, int w, const Geo& g, int i, int j) {
  Taps t;
  t.zero = g.pw <= 0 || g.ph <= 0 || j < g.zx || i < g.zy;
  const int ii = i - g.zy, jj = j - g.zx;
  const bool same = (ii < g.ry || ii >= g.rh);
  const int row = g.base_row + max(0, min(ii, g.rh) - g.ry);
  const bool left = jj < g.rx, right = !left && jj >= g.rw;
  t.edge = left || right;
  const int ce = g.col0 + (left ? g.rx : g.rw);
  const int c0 = t.zero ? 0 : (t.edge ? ce : g.col0 + jj);
  const int c1 = t.zero ? 0 : (t.edge ? ce : g.col0 + jj + 1);
  const size_t r1 = t.zero ? 0 : (size_t)row * w;
  const size_t r2 = (t.zero || same) ? r1 : r1 + w;
  // image levels live in device global memory: global (not flat) loads, so the waits count vmcnt only
  const __attribute__((address_space(1))) float* gi = (const __attribute__((address_space(1))) float*)img;
  t.v11 = gi[r1 + c0];
  t.v12 = gi[r1 + c1];
  t.v21 = gi[r2 + c0];
  t.v22 = gi[r2 + c1];
  return t;
}
__device__ __forceinline__ float sample(const float* img, int w, const Geo& g, int i, int j) {
  return combine(taps_global(img, w, g, i, j), g);
}

// Staged sampling (Track's Newton probes): each wave copies a kStT x kStT tile of the destination level around
// its estimate into LDS and samples from it with sample()'s index arithmetic (the same floats, so the results
// are bit-identical) — an LDS round trip per probe batch instead of an L2 one.  The wave restages when the
// estimate comes within a patch half-width + 3 pixels of the tile edge; near the image border (or on levels
// smaller than the tile) it samples global memory as before.
constexpr int kStT = 40;

struct Stage {
  int r0 = 0, c0 = 0;
  bool on = false;
};

__device__ __forceinline__ Taps taps_lds(const float* tile, const Stage& st, const Geo& g, int i, int j) {
  Taps t;
  t.zero = g.pw <= 0 || g.ph <= 0 || j < g.zx || i < g.zy;
  const int ii = i - g.zy, jj = j - g.zx;
  const bool same = (ii < g.ry || ii >= g.rh);
  const int row = g.base_row + max(0, min(ii, g.rh) - g.ry);
  const bool left = jj < g.rx, right = !left && jj >= g.rw;
  t.edge = left || right;
  const int ce = g.col0 + (left ? g.rx : g.rw);
  const int c0 = t.zero ? 0 : (t.edge ? ce : g.col0 + jj) - st.c0;
  const int c1 = t.zero ? 0 : (t.edge ? ce : g.col0 + jj + 1) - st.c0;
  const int r1 = t.zero ? 0 : (row - st.r0) * kStT;
  const int r2 = (t.zero || same) ? r1 : r1 + kStT;
  t.v11 = tile[r1 + c0];
  t.v12 = tile[r1 + c1];
  t.v21 = tile[r2 + c0];
  t.v22 = tile[r2 + c1];
  return t;
}
__device__ __forceinline__ float sample_lds(const float* tile, const Stage& st, const Geo& g, int i, int j) {
  return combine(taps_lds(tile, st, g, i, j), g);
}

// Every tap of the six probes around (x, y) lies in the staged tile (wave-uniform): the probes' windows span
// columns floor(x -+ 0.02 - (W - 1) / 2) .. + W, rows likewise.
__device__ __forceinline__ bool stage_covers(const Stage& st, float x, float y, int W) {
  const float lo = 0.5f * W + 3.f, hi = kStT - 0.5f * W - 4.f;
  return st.on && x >= st.c0 + lo && x <= st.c0 + hi && y >= st.r0 + lo && y <= st.r0 + hi;
}

// (Re)stage the tile around (x, y); levels smaller than the tile are never staged.  Split in two so a caller
// can put the tile's loads in flight beside other loads (stage_issue), then write the tile (stage_commit).
constexpr int kStV = (kStT * kStT + 63) / 64;   // tile values per lane
__device__ __forceinline__ bool stage_issue(const LevelDev& L, float x, float y, int lane, float (&v)[kStV],
                                            Stage& st) {
  if (L.w < kStT || L.h < kStT) {
    st.on = false;
    return false;
  }
  st.c0 = min(max((int)x - kStT / 2, 0), L.w - kStT);
  st.r0 = min(max((int)y - kStT / 2, 0), L.h - kStT);
  const __attribute__((address_space(1))) float* gi = (const __attribute__((address_space(1))) float*)L.img;
#pragma unroll
  for (int u = 0; u < kStV; ++u) {
    const int idx = min(lane + 64 * u, kStT * kStT - 1);
    v[u] = gi[(size_t)(st.r0 + idx / kStT) * L.w + st.c0 + idx % kStT];
  }
  return true;
}
__device__ __forceinline__ void stage_commit(const float (&v)[kStV], int lane, float* tile, Stage& st) {
#pragma unroll
  for (int u = 0; u < kStV; ++u) {
    const int idx = lane + 64 * u;
    if (idx < kStT * kStT) tile[idx] = v[u];
  }
  __builtin_amdgcn_wave_barrier();
  st.on = true;
}
__device__ __forceinline__ void stage_load(const LevelDev& L, float x, float y, int lane, float* tile, Stage& st) {
  float v[kStV];
  if (stage_issue(L, x, y, lane, v, st)) stage_commit(v, lane, tile, st);
}

template <int kCtrl>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kCtrl, 0xF, 0xF, false));
}
__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// Pairwise tree over the 64 lane partials (the oracle's LaneTreeSum order).  All lanes active.
__device__ __forceinline__ float wave_tree_sum(float v) {
  v = v + dpp_f<0xB1>(v);    // lanes (l, l^1)
  v = v + dpp_f<0x4E>(v);    // (l, l^2)
  v = v + dpp_f<0x141>(v);   // half-row mirror: octets
  v = v + dpp_f<0x140>(v);   // row mirror: 16-lane rows
  // (row 0 + row 1) + (row 2 + row 3) by gfx950 row swaps, in every lane (addition commutes: the same bits as
  // the readlane form (r0 + r16) + (r32 + r48), three instructions fewer)
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float w = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(w), __float_as_uint(w), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// N tree sums at once, stage by stage (the wave_tree_sum order for each), so the DPP and row-swap latencies of one
// sum overlap the others' instead of running back to back with wait states between.
template <int N>
__device__ __forceinline__ void wave_tree_sums(float (&v)[N]) {
#pragma unroll
  for (int r = 0; r < N; ++r) v[r] = v[r] + dpp_f<0xB1>(v[r]);
#pragma unroll
  for (int r = 0; r < N; ++r) v[r] = v[r] + dpp_f<0x4E>(v[r]);
#pragma unroll
  for (int r = 0; r < N; ++r) v[r] = v[r] + dpp_f<0x141>(v[r]);
#pragma unroll
  for (int r = 0; r < N; ++r) v[r] = v[r] + dpp_f<0x140>(v[r]);
#pragma unroll
  for (int r = 0; r < N; ++r) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[r]), __float_as_uint(v[r]), false, false);
    v[r] = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  }
#pragma unroll
  for (int r = 0; r < N; ++r) {
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[r]), __float_as_uint(v[r]), false, false);
    v[r] = __uint_as_float(b[0]) + __uint_as_float(b[1]);
  }
}

struct Tmpl {
  float v[kNP];
  float mean, sumsq;
};

__device__ __forceinline__ void get_patch(const LevelDev& L, float px, float py, int W, int lane, Tmpl& t) {
  Geo g;
  make_geo(px, py, W, L.w, L.h, g);
  const int len = W * W;
  float s = 0.f, q = 0.f;
#pragma unroll
  for (int k = 0; k < kNP; ++k) {
    const int p = lane + 64 * k;
    const float sv = sample(L.img, L.w, g, p / W, p % W);   // unconditional: loads in flight together
    const float v = (p < len) ? sv : 0.f;
    t.v[k] = v;
    s += v;
    q += v * v;
  }
  s = wave_tree_sum(s);
  q = wave_tree_sum(q);
  t.mean = s / len;
  t.sumsq = q / len;
}

// Diagnostic per-phase cycle counters of the Newton loop (lane 0 of each wave; SG_TRK_STAMP=1), added to the
// tracker's stamp buffer at the end of the kernel.  `on` is wave-uniform: production launches branch past it.
struct TStamp {
  unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long last = 0;
  bool on = false;
  __device__ __forceinline__ void mark(int slot) {
    if (on) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      acc[slot] += now - last;
      last = now;
    }
  }
};

struct TrackCtx {
  int W, len, max_it;
  float lenf, rlen;    // len as a float and its correctly rounded reciprocal (div_const)
  int nk;              // patch pixels per lane actually used: ceil(len / 64) <= kNP
  float threshold;
  int lane;
  float mk[kNP];       // this lane's mask values
  int pi[kNP], pj[kNP];   // this lane's patch pixels (row, column); pi = -1 past the patch
  TStamp* ts = nullptr;
};

// NK: patch pixels per lane the launch's window needs, ceil(W^2 / 64) (the kernels are instantiated per NK:
// slots past the patch only ever add zeros, so skipping them changes no bit and saves their sampling — at
// W = 7 three of the four slots).
template <int NK>
__device__ __forceinline__ void get_patch_ctx(const TrackCtx& c, const LevelDev& L, float px, float py, Tmpl& t) {
  Geo g;
  make_geo(px, py, c.W, L.w, L.h, g);
  float s = 0.f, q = 0.f;
#pragma unroll
  for (int k = 0; k < kNP; ++k) t.v[k] = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const float v = k < c.nk ? sample(L.img, L.w, g, c.pi[k], c.pj[k]) : 0.f;   // 0 past the patch
    t.v[k] = v;
    s += v;
    q += v * v;
  }
  s = wave_tree_sum(s);
  q = wave_tree_sum(q);
  t.mean = s / c.len;
  t.sumsq = q / c.len;
}

// Division by a constant divisor without the division sequence (Markstein): q0 = x r with r = RN(1 / b), the
// residual x - q0 b exact by one FMA, one correction q0 + (x - q0 b) r: the correctly rounded quotient x / b for
// every finite, normal x when r is the correctly rounded reciprocal (tests/test_const_division.py checks it on
// random operands for the tracker's divisors; infinities pass through as x r).  Three instructions instead of a
// correctly rounded division's eleven dependent ones, the same bits.
__device__ __forceinline__ double div_const(double x, double b, double r) {
  const double q0 = x * r;
  const double q = fma(fma(-q0, b, x), r, q0);
  return isinf(x) ? q0 : q;
}
__device__ __forceinline__ float div_const(float x, float b, float r) {
  const float q0 = x * r;
  const float q = fmaf(fmaf(-q0, b, x), r, q0);
  return isinf(x) ? q0 : q;
}

// BruteHessian (hessian.h:147-172): the six probes sampled together, their sums reduced in batches.
// kLds: the probes read the wave's staged tile (the caller checked stage_covers).
template <int NK, bool kLds>
__device__ __forceinline__ void brute_hessian(const TrackCtx& c, const LevelDev& L, const Tmpl& tp, float x, float y,
                                              float* mdx, float* mdy, float* mdxx, float* mdxy, float* mdyx,
                                              float* mdyy, const float* tile, const Stage& st) {
  c.ts->mark(0);
  const double hh = 0.02;
  // probes: sad0 (x, y), sadn1x (x - h, y), sadn1y (x, y - h), sadp1x (x + h, y), sadp1y (x, y + h), sadxy
  // (x + h, y + h).  Their column geometry is one of three (x, x - h, x + h), the row geometry one of three.
  // The three column and three row geometries are formed on lanes 0-2 (lane v: x, x - h, x + h and y, y - h,
  // y + h: the same float operations, so the same values) and broadcast by readlane.
  const int v = min(c.lane, 2);
  const float xv = v == 0 ? x : (float)(v == 1 ? x - hh : x + hh);
  const float yv = v == 0 ? y : (float)(v == 1 ? y - hh : y + hh);
  GeoX lx;
  GeoY ly;
  make_geo_x(xv, c.W, L.w, lx);
  make_geo_y(yv, c.W, L.h, ly);
  // variant 0's integer geometry to every lane; lanes 1 and 2 compare theirs with it (one ballot).  The five
  // integers of each half travel as one packed word (zx, rx, rw: 0..W <= 16, 5 bits each; col0: 17 signed bits;
  // pw = W - zx), so two readlanes and one compare per half instead of ten and five
  const unsigned pkx = (unsigned)lx.zx | ((unsigned)lx.rx << 5) | ((unsigned)lx.rw << 10) | ((unsigned)lx.col0 << 15);
  const unsigned pky = (unsigned)ly.zy | ((unsigned)ly.ry << 5) | ((unsigned)ly.rh << 10) |
                       ((unsigned)ly.base_row << 15);
  const unsigned px0 = __builtin_amdgcn_readfirstlane(pkx), py0 = __builtin_amdgcn_readfirstlane(pky);
  GeoX gx0;
  GeoY gy0;
  gx0.zx = (int)(px0 & 31u);
  gx0.pw = c.W - gx0.zx;
  gx0.rx = (int)((px0 >> 5) & 31u);
  gx0.rw = (int)((px0 >> 10) & 31u);
  gx0.col0 = (int)px0 >> 15;
  gy0.zy = (int)(py0 & 31u);
  gy0.ph = c.W - gy0.zy;
  gy0.ry = (int)((py0 >> 5) & 31u);
  gy0.rh = (int)((py0 >> 10) & 31u);
  gy0.base_row = (int)py0 >> 15;
  float av[3], bv[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    av[u] = readlane_f(lx.a, u);
    bv[u] = readlane_f(ly.b, u);
  }
  gx0.a = av[0];
  gy0.b = bv[0];
  constexpr int kXi[6] = {0, 1, 0, 2, 0, 2}, kYi[6] = {0, 0, 1, 0, 2, 2};
  // Unless a probe crosses a pixel boundary (or the border), the six share their integer geometry and so every
  // tap: the taps are read once and combined with each probe's weights — the same floats as six samples.
  const bool same = pkx == px0 && pky == py0;   // (the packing is one to one: geo_x_same && geo_y_same)
  const bool shared = (__ballot(same) & 7ull) == 7ull;
  float pv[6][NK], ps[6], pq[6];
  if (shared) {
    Geo g0;
    geo_join(gx0, gy0, g0);
#pragma unroll
    for (int r = 0; r < 6; ++r) ps[r] = pq[r] = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const Taps t = kLds ? taps_lds(tile, st, g0, c.pi[k], c.pj[k]) : taps_global(L.img, L.w, g0, c.pi[k], c.pj[k]);
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        Geo g = g0;
        const GeoX wx{0, 0, 0, 0, 0, av[kXi[r]]};
        const GeoY wy{0, 0, 0, 0, 0, bv[kYi[r]]};
        {
          Geo w;
          geo_join(wx, wy, w);   // the probe's weights (its integer fields are g0's)
          g.a11 = w.a11;
          g.a12 = w.a12;
          g.a21 = w.a21;
          g.a22 = w.a22;
          g.b1 = w.b1;
          g.b2 = w.b2;
        }
        const float v = combine_sel(t, g, k < c.nk);   // 0 past the patch
        pv[r][k] = v;
        ps[r] += v;
        pq[r] += v * v;
      }
    }
  } else {
    GeoX gx[3];
    GeoY gy[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      gx[u].zx = __builtin_amdgcn_readlane(lx.zx, u);
      gx[u].pw = __builtin_amdgcn_readlane(lx.pw, u);
      gx[u].col0 = __builtin_amdgcn_readlane(lx.col0, u);
      gx[u].rx = __builtin_amdgcn_readlane(lx.rx, u);
      gx[u].rw = __builtin_amdgcn_readlane(lx.rw, u);
      gx[u].a = av[u];
      gy[u].zy = __builtin_amdgcn_readlane(ly.zy, u);
      gy[u].ph = __builtin_amdgcn_readlane(ly.ph, u);
      gy[u].base_row = __builtin_amdgcn_readlane(ly.base_row, u);
      gy[u].ry = __builtin_amdgcn_readlane(ly.ry, u);
      gy[u].rh = __builtin_amdgcn_readlane(ly.rh, u);
      gy[u].b = bv[u];
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      Geo g;
      geo_join(gx[kXi[r]], gy[kYi[r]], g);
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        const float sv = kLds ? sample_lds(tile, st, g, c.pi[k], c.pj[k]) : sample(L.img, L.w, g, c.pi[k], c.pj[k]);
        const float v = k < c.nk ? sv : 0.f;   // 0 past the patch
        pv[r][k] = v;
        s += v;
        q += v * v;
      }
      ps[r] = s;
      pq[r] = q;
    }
  }
  c.ts->mark(1);
  // The twelve tree sums (wave_tree_sum's order for each): the four DPP stages per value, then the two row stages
  // for a probe's pair (ps, pq) at once — one row swap puts ps's rows 0 + 1 / 2 + 3 in rows 0 / 2 and pq's in rows
  // 1 / 3 (the same additions, so the same bits), and the last swap finishes both: ps's total in rows 0 and 2,
  // pq's in rows 1 and 3.  Half the row-swap instructions of twelve separate sums.
  float tot[6];
  {
    float sums[12];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      sums[r] = ps[r];
      sums[6 + r] = pq[r];
    }
#pragma unroll
    for (int r = 0; r < 12; ++r) sums[r] = sums[r] + dpp_f<0xB1>(sums[r]);
#pragma unroll
    for (int r = 0; r < 12; ++r) sums[r] = sums[r] + dpp_f<0x4E>(sums[r]);
#pragma unroll
    for (int r = 0; r < 12; ++r) sums[r] = sums[r] + dpp_f<0x141>(sums[r]);
#pragma unroll
    for (int r = 0; r < 12; ++r) sums[r] = sums[r] + dpp_f<0x140>(sums[r]);
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(sums[r]), __float_as_uint(sums[6 + r]), false,
                                                      false);
      tot[r] = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(tot[r]), __float_as_uint(tot[r]), false, false);
      tot[r] = __uint_as_float(b[0]) + __uint_as_float(b[1]);
    }
  }
  c.ts->mark(2);
  // each probe's lighting fit (ScorePatchMatch, hessian.h:131-133: mean, second moment, alpha, beta) on its own
  // lane (probe = lane, 0..5; the same float operations, so the same bits) and broadcast by readlane: one chain
  // of three divisions and a square root in the instruction stream instead of six
  float alphas[6], betas[6];
  {
    // probe r's ps total from lane r (row 0), its pq total from lane 16 + r (row 1), moved to row 0 by one swap
    const int r = min(c.lane & 15, 5);
    const float psl = r == 0 ? tot[0] : r == 1 ? tot[1] : r == 2 ? tot[2] : r == 3 ? tot[3] : r == 4 ? tot[4] : tot[5];
    const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(psl), __float_as_uint(psl), false, false);
    const float pql = __uint_as_float(sw[1]);
    const float mean = div_const(psl, c.lenf, c.rlen), sumsq = div_const(pql, c.lenf, c.rlen);   // psl / len, pql / len
    const float alpha = sqrtf(tp.sumsq / sumsq);
    const float beta = tp.mean - alpha * mean;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      alphas[q] = readlane_f(alpha, q);
      betas[q] = readlane_f(beta, q);
    }
  }
  float sc[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const float alpha = alphas[r], beta = betas[r];
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      float term = 0.f;
      const float a = tp.v[k], b = pv[r][k];
      if (!(a == 0 || b == 0)) {
        float diff = a - b * alpha - beta;
        diff = diff * diff;
        term = diff * c.mk[k];
      }
      acc += term;
    }
    sc[r] = acc;
  }
  c.ts->mark(3);
  // the six score sums as the probe sums above: DPP stages per value, the row stages per pair (sc[2k] ends in rows
  // 0 / 2, sc[2k+1] in rows 1 / 3, brought to row 0 by one more swap); the quotient lanes 0-5 are in row 0
#pragma unroll
  for (int r = 0; r < 6; ++r) sc[r] = sc[r] + dpp_f<0xB1>(sc[r]);
#pragma unroll
  for (int r = 0; r < 6; ++r) sc[r] = sc[r] + dpp_f<0x4E>(sc[r]);
#pragma unroll
  for (int r = 0; r < 6; ++r) sc[r] = sc[r] + dpp_f<0x141>(sc[r]);
#pragma unroll
  for (int r = 0; r < 6; ++r) sc[r] = sc[r] + dpp_f<0x140>(sc[r]);
  float sct[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(sc[2 * k]), __float_as_uint(sc[2 * k + 1]), false,
                                                    false);
    sct[k] = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(sct[k]), __float_as_uint(sct[k]), false, false);
    sct[k] = __uint_as_float(b[0]) + __uint_as_float(b[1]);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const auto o = __builtin_amdgcn_permlane16_swap(__float_as_uint(sct[k]), __float_as_uint(sct[k]), false, false);
    sc[2 * k] = sct[k];                      // (row 0)
    sc[2 * k + 1] = __uint_as_float(o[1]);  // row 1's total, in row 0
  }
  const double sad0 = sc[0], sadn1x = sc[1], sadn1y = sc[2], sadp1x = sc[3], sadp1y = sc[4], sadxy = sc[5];
  // The six difference quotients of hessian.h:160-171, one per lane (lane e computes quotient e with the
  // reference's fp64 operations in the reference's order, so the bits are the same) and gathered by readlane:
  // three fp64 divisions in the wave's instruction stream instead of fourteen (a correctly rounded fp64
  // division is about eleven dependent instructions).
  //   e 0: mdx = 0.5 (p1x - n1x) / h        e 2: mdxx = ((p1x - s0) / h - (s0 - n1x) / h) / h
  //   e 1: mdy = 0.5 (p1y - n1y) / h        e 3: mdyy = ((p1y - s0) / h - (s0 - n1y) / h) / h
  //                                         e 4: mdxy = ((sxy - p1y) / h - (p1x - s0) / h) / h
  //                                         e 5: mdyx = ((sxy - p1x) / h - (p1y - s0) / h) / h
  const int e = c.lane;
  const double qa = e == 0 ? sadp1x : e == 1 ? sadp1y : e == 2 ? sadp1x : e == 3 ? sadp1y : sadxy;
  const double qb = e == 0 ? sadn1x : e == 1 ? sadn1y : e == 2 || e == 3 ? sad0 : e == 4 ? sadp1y : sadp1x;
  const double qc = e == 2 || e == 3 ? sad0 : e == 4 ? sadp1x : sadp1y;
  const double qd = e == 2 ? sadn1x : e == 3 ? sadn1y : sad0;
  const double num = e < 2 ? 0.5 * (qa - qb) : (qa - qb);
  constexpr double rh = 50.0;   // RN(1 / 0.02): the quotients by h as div_const (the same bits as "/ hh")
  const double q1 = div_const(num, hh, rh);
  const double q2 = div_const(qc - qd, hh, rh);
  const float res = (float)(e < 2 ? q1 : div_const(q1 - q2, hh, rh));
  *mdx = readlane_f(res, 0);
  *mdy = readlane_f(res, 1);
  *mdxx = readlane_f(res, 2);
  *mdyy = readlane_f(res, 3);
  *mdxy = readlane_f(res, 4);
  *mdyx = readlane_f(res, 5);
  c.ts->mark(4);
}

// One TrackFeature (hessian.h:243-264) pass: templates from `src` at (sx, sy) (GetPatches, 175-183), Newton
// iterations of Track (185-241) on `dst` coarse to fine.  0 OK (*px, *py updated), 2 OUT_OF_BOUNDS.
template <int NK>
__device__ __forceinline__ int track_pass(const TrackCtx& c, const LevelDev* __restrict__ src,
                                          const LevelDev* __restrict__ dst, int lvls, float sx, float sy, float* px,
                                          float* py, int* iters, float* tile) {
  const double s = 1. / (1 << (lvls - 1));
  float x = (float)(*px * s), y = (float)(*py * s);
  for (int i = lvls - 1; i >= 0; --i) {
    float tx = sx, ty = sy;
    for (int k = 0; k < i; ++k) {
      tx = (float)(tx * 0.5);
      ty = (float)(ty * 0.5);
    }
    const LevelDev Ls = src[i], Ld = dst[i];
    Tmpl tp;
    c.ts->mark(7);
    // the destination tile around the level's start estimate and the template patch: both sets of loads in
    // flight together (one memory round trip per level instead of two); the tile is the one the first Newton
    // iteration would stage (same values: the probes sample identical floats from it or from global memory)
    Stage st;
    float sv[kStV];
    const bool pre = stage_issue(Ld, x, y, c.lane, sv, st);
    get_patch_ctx<NK>(c, Ls, tx, ty, tp);
    if (pre) stage_commit(sv, c.lane, tile, st);
#ifdef SG_X_DUPSTART   // timing-only A/B (tools/r5_trk_ab.sh): the level start's fetches done twice
    {
      float xo = x, yo = y, txo = tx, tyo = ty;
      asm volatile("" : "+v"(xo), "+v"(yo), "+v"(txo), "+v"(tyo));
      Tmpl tp2;
      Stage st2 = st;
      const bool pre2 = stage_issue(Ld, xo, yo, c.lane, sv, st2);
      get_patch_ctx<NK>(c, Ls, txo, tyo, tp2);
      if (pre2) stage_commit(sv, c.lane, tile, st2);
      asm volatile("" ::"v"(tp2.mean), "v"(tp2.sumsq), "v"(tp2.v[0]));
    }
#endif
    c.ts->mark(6);
    const float margin = 0.01f;
    int it = 0;
    bool oob = false;
    for (; it < c.max_it; ++it) {
      if (x < margin || y < margin || (x + margin) > Ld.w || (y + margin) > Ld.h) {
        oob = true;
        break;
      }
      float mdx, mdy, mdxx, mdxy, mdyx, mdyy;
      if (!stage_covers(st, x, y, c.W)) stage_load(Ld, x, y, c.lane, tile, st);
      if (stage_covers(st, x, y, c.W))
        brute_hessian<NK, true>(c, Ld, tp, x, y, &mdx, &mdy, &mdxx, &mdxy, &mdyx, &mdyy, tile, st);
      else
        brute_hessian<NK, false>(c, Ld, tp, x, y, &mdx, &mdy, &mdxx, &mdxy, &mdyx, &mdyy, tile, st);
#ifdef SG_X_DUPITER   // timing-only A/B: every Newton iteration's probes and sums done twice
      {
        float xo = x, yo = y, d0, d1, d2, d3, d4, d5;
        asm volatile("" : "+v"(xo), "+v"(yo));
        if (stage_covers(st, xo, yo, c.W))
          brute_hessian<NK, true>(c, Ld, tp, xo, yo, &d0, &d1, &d2, &d3, &d4, &d5, tile, st);
        else
          brute_hessian<NK, false>(c, Ld, tp, xo, yo, &d0, &d1, &d2, &d3, &d4, &d5, tile, st);
        asm volatile("" ::"v"(d0), "v"(d1), "v"(d2), "v"(d3), "v"(d4), "v"(d5));
      }
#endif
      const double H00 = mdxx, H01 = mdxy, H10 = mdyx, H11 = mdyy;
      const double det = H00 * H11 - H10 * H01;
      const double invdet = 1.0 / det;
      const double i00 = H11 * invdet, i10 = -H10 * invdet, i01 = -H01 * invdet, i11 = H00 * invdet;
      const double g0 = mdx, g1 = mdy;
      const double jj0 = i00 * g0 + i01 * g1, jj1 = i10 * g0 + i11 * g1;
      float dx = (float)-jj0, dy = (float)-jj1;
      if ((dx * dx + dy * dy) > 1) {
        dx /= sqrtf(dx * dx + dy * dy);
        dy /= sqrtf(dx * dx + dy * dy);   // with the updated dx, as the reference
      }
      const float cx = (dx < 1.f) ? dx : 1.f, cy = (dy < 1.f) ? dy : 1.f;   // std::min / std::max semantics
      x += (-1.f < cx) ? cx : -1.f;
      y += (-1.f < cy) ? cy : -1.f;
      c.ts->mark(5);
      if (fabsf(dx) < c.threshold && fabsf(dy) < c.threshold) {
        ++it;
        break;
      }
    }
    *iters += it;
    if (oob) return 2;
    if (i > 0) {
      x = (float)(x * 2.);
      y = (float)(y * 2.);
    }
  }
  *px = x;
  *py = y;
  return 0;
}

// matcher.cpp TrackFeature (173-206) + FindMatches' retry with more levels (247-251) of one feature (one wave):
// forward from (fx, fy) starting at (*tx, *ty), backward, the forward/backward check; *tx, *ty hold the last
// forward result (the retry starts from the forward-mutated to_pt, matcher.cpp:176, 247-248).  The backward pass
// is skipped when the forward pass failed: the matcher rejects the feature either way and the backward pass
// does not touch to_pt.
template <int NK>
__device__ __forceinline__ bool fb_track(const TrackCtx& c, const LevelDev* __restrict__ from_lv,
                                         const LevelDev* __restrict__ to_lv, int depth, const TrackParams& prm,
                                         float fx, float fy, int lv0, float* ptx, float* pty, int* piters,
                                         float* tile) {
  float tx = *ptx, ty = *pty;
  int iters = *piters;
  bool ok = false;
  for (int attempt = 0; attempt < 2 && !ok; ++attempt) {
    int lv = lv0;
    if (attempt == 1) {
      if (prm.retry_levels <= 0 || lv0 == prm.retry_levels) break;
      lv = prm.retry_levels;
    }
    const int lvls = min(depth, lv);
    int st = 0;
    float bx = fx, by = fy;
    for (int pass = 0; pass < 2; ++pass) {
      const LevelDev* src = pass ? to_lv : from_lv;
      const LevelDev* dst = pass ? from_lv : to_lv;
      const float sx = pass ? tx : fx, sy = pass ? ty : fy;
      float qx = pass ? bx : tx, qy = pass ? by : ty;
      st = track_pass<NK>(c, src, dst, lvls, sx, sy, &qx, &qy, &iters, tile);
      if (st != 0) break;
      if (pass == 0) {
        tx = qx;
        ty = qy;
      } else {
        bx = qx;
        by = qy;
      }
    }
    if (st == 0) {
      const float ex = fx - bx, ey = fy - by;
      ok = !(sqrt((double)ex * ex + (double)ey * ey) > (double)prm.fb_max);
    }
  }
  *ptx = tx;
  *pty = ty;
  *piters = iters;
  return ok;
}

__device__ __forceinline__ void init_ctx(TrackCtx& c, const TrackParams& prm, int lane);

// matcher.cpp TrackFeature (173-206) + FindMatches' retry with more levels (247-251), one wave per feature.
template <int NK>
__global__ __launch_bounds__(64 * kTrackWaves) void k_track_fb(const LevelDev* __restrict__ from_lv,
                                                               const LevelDev* __restrict__ to_lv, int depth,
                                                               TrackParams prm, int n, const float* from_xy,
                                                               const float* to_init, const int32_t* levels,
                                                               float* to_xy, int32_t* accepted, int32_t* iterations) {
  __shared__ float stage_tiles[kTrackWaves][kStT * kStT];
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * kTrackWaves + (threadIdx.x >> 6);
  if (f >= n) return;   // whole wave
  float* tile = stage_tiles[threadIdx.x >> 6];
  TStamp tst;
  tst.on = prm.stamps != nullptr && lane == 0;
  if (tst.on) tst.last = __builtin_amdgcn_s_memtime();
  TrackCtx c;
  c.ts = &tst;
  c.W = prm.window;
  c.len = prm.window * prm.window;
  c.lenf = (float)c.len;
  c.rlen = 1.0f / c.lenf;
  c.nk = (c.len + 63) / 64;
  c.max_it = prm.max_iterations;
  c.threshold = prm.threshold;
  c.lane = lane;
#pragma unroll
  for (int k = 0; k < kNP; ++k) {
    const int p = lane + 64 * k;
    const bool in = p < c.len;
    c.mk[k] = in ? prm.mask[p] : 0.f;
    c.pi[k] = in ? p / c.W : -1;
    c.pj[k] = in ? p % c.W : 0;
  }
  const float fx = from_xy[2 * f], fy = from_xy[2 * f + 1];
  float tx = to_init[2 * f], ty = to_init[2 * f + 1];
  const int lv0 = levels ? levels[f] : 3;
  int iters = 0;
  const bool ok = fb_track<NK>(c, from_lv, to_lv, depth, prm, fx, fy, lv0, &tx, &ty, &iters, tile);
  if (lane == 0) {
    to_xy[2 * f] = tx;
    to_xy[2 * f + 1] = ty;
    accepted[f] = ok ? 1 : 0;
    if (iterations) iterations[f] = iters;
  }
  if (tst.on) {
    tst.mark(7);
    for (int k = 0; k < 8; ++k) atomicAdd(prm.stamps + k, tst.acc[k]);
    atomicAdd(prm.stamps + 8, (unsigned long long)iters);
    atomicAdd(prm.stamps + 9, 1ull);
  }
}

__global__ __launch_bounds__(64 * kTrackWaves) void k_get_patches(LevelDev L, int W, int n, const float* xy, float* out,
                                                                  float* mean, float* sumsq) {
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * kTrackWaves + (threadIdx.x >> 6);
  if (f >= n) return;
  Tmpl t;
  get_patch(L, xy[2 * f], xy[2 * f + 1], W, lane, t);
  const int len = W * W;
#pragma unroll
  for (int k = 0; k < kNP; ++k) {
    const int p = lane + 64 * k;
    if (p < len) out[(size_t)f * len + p] = t.v[k];
  }
  if (lane == 0) {
    mean[f] = t.mean;
    sumsq[f] = t.sumsq;
  }
}

// ------------------------------------------------------------------------------------------------
// One-directional TrackFeature of each FeatureTracker (sg_tracker_track_feature).

__device__ __forceinline__ void init_ctx(TrackCtx& c, const TrackParams& prm, int lane) {
  // (the one-directional kernels are not stamped: c.ts points at an off TStamp set by the caller)
  c.W = prm.window;
  c.len = prm.window * prm.window;
  c.lenf = (float)c.len;
  c.rlen = 1.0f / c.lenf;
  c.nk = (c.len + 63) / 64;
  c.max_it = prm.max_iterations;
  c.threshold = prm.threshold;
  c.lane = lane;
#pragma unroll
  for (int k = 0; k < kNP; ++k) {
    const int p = lane + 64 * k;
    const bool in = p < c.len;
    c.mk[k] = in ? prm.mask[p] : 0.f;
    c.pi[k] = in ? p / c.W : -1;
    c.pj[k] = in ? p % c.W : 0;
  }
}

// HessianTracker::TrackFeature (hessian.h:243-264) alone, one wave per feature.
template <int NK>
__global__ __launch_bounds__(64 * kTrackWaves) void k_track_one(const LevelDev* __restrict__ from_lv,
                                                                const LevelDev* __restrict__ to_lv, int depth,
                                                                TrackParams prm, int n, const float* from_xy,
                                                                float* to_xy, const int32_t* levels,
                                                                int32_t* status, int32_t* iterations) {
  __shared__ float stage_tiles[kTrackWaves][kStT * kStT];
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * kTrackWaves + (threadIdx.x >> 6);
  if (f >= n) return;
  float* tile = stage_tiles[threadIdx.x >> 6];
  TrackCtx c;
  TStamp tst_off;
  init_ctx(c, prm, lane);
  c.ts = &tst_off;
  const int lvls = min(depth, levels ? levels[f] : depth);
  float qx = to_xy[2 * f], qy = to_xy[2 * f + 1];
  int iters = 0;
  const int st = track_pass<NK>(c, from_lv, to_lv, lvls, from_xy[2 * f], from_xy[2 * f + 1], &qx, &qy, &iters, tile);
  if (lane == 0) {
    status[f] = st;
    if (st == 0) {
      to_xy[2 * f] = qx;
      to_xy[2 * f + 1] = qy;
    }
    if (iterations) iterations[f] = iters;
  }
}

// matcher.cpp FindMatches (210-271) over a batch of features into one view: one wave per feature walks the
// feature's attempts — a stored view (pyramid slot) and its match point, the starting point in the new view, in
// the feature's view order, out-of-bounds starts already dropped (matcher.cpp:245-247) — and stops at the first
// forward/backward-consistent track (fb_track, with the retry).  which[f]: the accepted attempt (-1: none), to_xy
// its track.  A frame's matching is one launch instead of a host round trip per view and round.
template <int NK>
__global__ __launch_bounds__(64 * kTrackWaves) void k_find_matches(const LevelDev* __restrict__ tabs, int to_slot,
                                                                   int depth, TrackParams prm, int n,
                                                                   const int32_t* __restrict__ aoff,
                                                                   const int32_t* __restrict__ aslot,
                                                                   const float4* __restrict__ axy,
                                                                   const int32_t* __restrict__ levels, float* to_xy,
                                                                   int32_t* which, int32_t* iterations) {
  __shared__ float stage_tiles[kTrackWaves][kStT * kStT];
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * kTrackWaves + (threadIdx.x >> 6);
  if (f >= n) return;   // whole wave
  float* tile = stage_tiles[threadIdx.x >> 6];
  TrackCtx c;
  TStamp tst_off;
  init_ctx(c, prm, lane);
  c.ts = &tst_off;
  const LevelDev* to_lv = tabs + (size_t)to_slot * kTrkMaxDepth;
  const int a0 = aoff[f], a1 = aoff[f + 1], lv0 = levels[f];
  int iters = 0, hit = -1;
  float tx = 0.f, ty = 0.f;
  for (int a = a0; a < a1 && hit < 0; ++a) {
    const float4 xy = axy[a];
    tx = xy.z;
    ty = xy.w;
    if (fb_track<NK>(c, tabs + (size_t)aslot[a] * kTrkMaxDepth, to_lv, depth, prm, xy.x, xy.y, lv0, &tx, &ty, &iters,
                     tile))
      hit = a - a0;
  }
  if (lane == 0) {
    to_xy[2 * f] = tx;
    to_xy[2 * f + 1] = ty;
    which[f] = hit;
    if (iterations) iterations[f] = iters;
  }
}

// klt.h BruteHessian (181-204): forward differences (h = 0.01) of SADPatches(template, probe) (139-149), the
// masked, not lighting-normalised SSD, on plain getRectSubPix probes; six probes sampled together.
__device__ __forceinline__ void klt_hessian(const TrackCtx& c, const LevelDev& L, const Tmpl& tp, float x, float y,
                                            float* mdx, float* mdy, float* mdxx, float* mdxy, float* mdyx,
                                            float* mdyy) {
  const double hh = 0.01;
  float px[6], py[6];
  px[0] = x;                   py[0] = y;                    // sad0
  px[1] = (float)(x + hh);     py[1] = y;                    // sadx
  px[2] = x;                   py[2] = (float)(y + hh);      // sady
  px[3] = (float)(x + 2 * hh); py[3] = y;                    // sadxx
  px[4] = x;                   py[4] = (float)(y + 2 * hh);  // sadyy
  px[5] = (float)(x + hh);     py[5] = (float)(y + hh);      // sadxy
  float sc[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    Geo g;
    make_geo<false>(px[r], py[r], c.W, L.w, L.h, g);
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < kNP; ++k) {
      float term = 0.f;
      if (c.pi[k] >= 0) {
        const float a = tp.v[k], b = sample(L.img, L.w, g, c.pi[k], c.pj[k]);
        if (!(a == 0 || b == 0)) {
          const float diff = a - b;
          term = diff * diff * c.mk[k];
        }
      }
      acc += term;
    }
    sc[r] = acc;
  }
#pragma unroll
  for (int r = 0; r < 6; ++r) sc[r] = wave_tree_sum(sc[r]);
  const double sad0 = sc[0], sadx = sc[1], sady = sc[2], sadxx = sc[3], sadyy = sc[4], sadxy = sc[5];
  *mdx = (float)((sadx - sad0) / hh);
  *mdy = (float)((sady - sad0) / hh);
  *mdxx = (float)(((sadxx - sadx) / hh - (sadx - sad0) / hh) / hh);
  *mdyy = (float)(((sadyy - sady) / hh - (sady - sad0) / hh) / hh);
  *mdxy = (float)(((sadxy - sady) / hh - (sadx - sad0) / hh) / hh);
  *mdyx = (float)(((sadxy - sadx) / hh - (sady - sad0) / hh) / hh);
}

// klt.h:258-401 Track (the LK matrices A, B, C, RS, VW it accumulates are overwritten by the BruteHessian step
// before use, so they are not formed): margin 0.1, stop when both steps are below threshold / 10.
__device__ __forceinline__ int klt_track(const TrackCtx& c, const LevelDev& L, const Tmpl& tp, float threshold,
                                         float* px, float* py, int* iters) {
  float x = *px, y = *py;
  const float margin = 0.1f;
  int it = 0;
  for (; it < c.max_it; ++it) {
    if (x < margin || y < margin || (x + margin) > L.w || (y + margin) > L.h) {
      *iters += it;
      return 2;
    }
    float mdx, mdy, mdxx, mdxy, mdyx, mdyy;
    klt_hessian(c, L, tp, x, y, &mdx, &mdy, &mdxx, &mdxy, &mdyx, &mdyy);
    const double H00 = mdxx, H01 = mdxy, H10 = mdyx, H11 = mdyy;
    const double det = H00 * H11 - H10 * H01;
    const double invdet = 1.0 / det;
    const double i00 = H11 * invdet, i10 = -H10 * invdet, i01 = -H01 * invdet, i11 = H00 * invdet;
    const double g0 = mdx, g1 = mdy;
    const double jj0 = i00 * g0 + i01 * g1, jj1 = i10 * g0 + i11 * g1;
    float dx = (float)-jj0, dy = (float)-jj1;
    if ((dx * dx + dy * dy) > 1) {
      dx /= sqrtf(dx * dx + dy * dy);
      dy /= sqrtf(dx * dx + dy * dy);
    }
    const float cx = (dx < 1.f) ? dx : 1.f, cy = (dy < 1.f) ? dy : 1.f;
    x += (-1.f < cx) ? cx : -1.f;
    y += (-1.f < cy) ? cy : -1.f;
    if ((double)fabsf(dx) < threshold / 10. && (double)fabsf(dy) < threshold / 10.) {
      ++it;
      break;
    }
  }
  *iters += it;
  *px = x;
  *py = y;
  return 0;
}

// klt.h:403-424 TrackFeature, one wave per feature: every level, threshold x 50 on the coarse levels.
__global__ __launch_bounds__(64 * kTrackWaves) void k_track_klt(const LevelDev* __restrict__ from_lv,
                                                                const LevelDev* __restrict__ to_lv, int depth,
                                                                TrackParams prm, int n, const float* from_xy,
                                                                float* to_xy, int32_t* status, int32_t* iterations) {
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * kTrackWaves + (threadIdx.x >> 6);
  if (f >= n) return;
  TrackCtx c;
  TStamp tst_off;
  init_ctx(c, prm, lane);
  c.ts = &tst_off;
  const float sx = from_xy[2 * f], sy = from_xy[2 * f + 1];
  const double s = 1. / (1 << (depth - 1));
  float x = (float)(to_xy[2 * f] * s), y = (float)(to_xy[2 * f + 1] * s);
  int iters = 0, st = 0;
  for (int i = depth - 1; i >= 0; --i) {
    float tx = sx, ty = sy;
    for (int k = 0; k < i; ++k) {
      tx = (float)(tx * 0.5);
      ty = (float)(ty * 0.5);
    }
    const LevelDev Ls = from_lv[i];
    Geo g;
    make_geo<false>(tx, ty, c.W, Ls.w, Ls.h, g);
    Tmpl tp;
#pragma unroll
    for (int k = 0; k < kNP; ++k) tp.v[k] = c.pi[k] >= 0 ? sample(Ls.img, Ls.w, g, c.pi[k], c.pj[k]) : 0.f;
    st = klt_track(c, to_lv[i], tp, i > 0 ? prm.threshold * 50 : prm.threshold, &x, &y, &iters);
    if (st) break;
    if (i > 0) {
      x = (float)(x * 2.);
      y = (float)(y * 2.);
    }
  }
  if (lane == 0) {
    status[f] = st;
    if (st == 0) {
      to_xy[2 * f] = x;
      to_xy[2 * f + 1] = y;
    }
    if (iterations) iterations[f] = iters;
  }
}

// ---- brute.h (one thread per search candidate) --------------------------------------------------
constexpr int kBruteThreads = 256;

struct BruteState {
  float x, y;     // the search centre p (brute.h:143), at the current level's scale
  float sad;      // SearchBest's return value of the last pass
  int status;     // 0 tracking, 2 OUT_OF_BOUNDS
};

// GetPatch (brute.h:35-58: plain getRectSubPix, sequential sums) of one candidate and SADPatches(template,
// candidate) (82-94: lighting-normalised, unmasked, sequential sum).  The patch is sampled twice (sums, then
// the score) instead of being held in registers.
__device__ __forceinline__ float brute_candidate(const LevelDev& L, int W, const float* tmpl, float tmean,
                                                 float tsumsq, float px, float py) {
  Geo g;
  make_geo<false>(px, py, W, L.w, L.h, g);
  const int len = W * W;
  float sum = 0.f, sum_sq = 0.f;
  for (int i = 0; i < W; ++i)
    for (int j = 0; j < W; ++j) {
      const float d = sample(L.img, L.w, g, i, j);
      sum += d;
      sum_sq += d * d;
    }
  const float mean = sum / len, sumsq = sum_sq / len;
  const float alpha = sqrtf(tsumsq / sumsq);
  const float beta = tmean - alpha * mean;
  float acc = 0.f;
  for (int i = 0; i < W; ++i)
    for (int j = 0; j < W; ++j) {
      const float a = tmpl[i * W + j], d = sample(L.img, L.w, g, i, j);
      if (a == 0 || d == 0) continue;
      const float diff = a - d * alpha - beta;
      acc += fabsf(diff * diff);
    }
  return acc;
}

// Templates GetPatches(from, from_xy) (brute.h:120-127), thread per (feature, level); initial margin test and
// search centre (brute.h:136-143), thread per feature.
__global__ void k_brute_setup(const LevelDev* __restrict__ from_lv, const LevelDev* __restrict__ to_lv, int depth,
                              int W, int n, const float* from_xy, const float* to_xy, float* tmpls, BruteState* stt) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * depth) return;
  const int f = t / depth, l = t % depth;
  float tx = from_xy[2 * f], ty = from_xy[2 * f + 1];
  for (int k = 0; k < l; ++k) {
    tx = (float)(tx * 0.5);
    ty = (float)(ty * 0.5);
  }
  const LevelDev L = from_lv[l];
  Geo g;
  make_geo<false>(tx, ty, W, L.w, L.h, g);
  const int len = W * W;
  float* o = tmpls + ((size_t)f * depth + l) * (len + 2);
  float sum = 0.f, sum_sq = 0.f;
  for (int i = 0; i < W; ++i)
    for (int j = 0; j < W; ++j) {
      const float d = sample(L.img, L.w, g, i, j);
      o[i * W + j] = d;
      sum += d;
      sum_sq += d * d;
    }
  o[len] = sum / len;
  o[len + 1] = sum_sq / len;
  if (l == 0) {
    const float px = to_xy[2 * f], py = to_xy[2 * f + 1];
    const float margin = 13;
    BruteState s;
    s.status = (px < margin || py < margin || (px + margin) > to_lv[0].w || (py + margin) > to_lv[0].h) ? 2 : 0;
    const double sc = 1. / (1 << (depth - 1));
    s.x = (float)(px * sc);
    s.y = (float)(py * sc);
    s.sad = 0.f;
    stt[f] = s;
  }
}

// (sad, candidate) order of SearchBest (brute.h:104-113): a candidate wins unless its score is larger, so the
// result is the last candidate with the smallest score.  NaN scores never win here.
__device__ __forceinline__ bool brute_better(float sa, int ia, float sb, int ib) {
  return sa < sb || (sa == sb && ia > ib);
}

// One SearchBest pass: every candidate of every live feature, one per thread; workgroup bests to bsad / bidx.
__global__ __launch_bounds__(kBruteThreads) void k_brute_eval(const LevelDev* __restrict__ to_lv, int lvl, int W,
                                                              int depth, const float* tmpls, const float* steps,
                                                              int ns, const BruteState* stt, float* bsad, int* bidx,
                                                              int nblk) {
  __shared__ float rs[kBruteThreads / 64];
  __shared__ int ri[kBruteThreads / 64];
  const int f = blockIdx.y;
  const BruteState s = stt[f];
  float best = INFINITY;
  int bi = -1;
  const int c = blockIdx.x * kBruteThreads + threadIdx.x;
  if (s.status == 0 && c < ns * ns) {
    const float ox = steps[c / ns], oy = steps[c % ns];
    const int len = W * W;
    const float* t = tmpls + ((size_t)f * depth + lvl) * (len + 2);
    const float sad = brute_candidate(to_lv[lvl], W, t, t[len], t[len + 1], s.x + ox, s.y + oy);
    if (sad == sad) {
      best = sad;
      bi = c;
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const float os = __shfl_xor(best, m);
    const int oi = __shfl_xor(bi, m);
    if (brute_better(os, oi, best, bi)) {
      best = os;
      bi = oi;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = best;
    ri[threadIdx.x >> 6] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBruteThreads / 64; ++w)
      if (brute_better(rs[w], ri[w], best, bi)) {
        best = rs[w];
        bi = ri[w];
      }
    bsad[(size_t)f * nblk + blockIdx.x] = best;
    bidx[(size_t)f * nblk + blockIdx.x] = bi;
  }
}

// The pass's winner per feature (one wave each): p moves to it when its score is <= SearchBest's initial 1e6;
// check: sad > 100 -> OUT_OF_BOUNDS (brute.h:147-148, 158-159); scale: p *= 2 for the next level.
__global__ void k_brute_pick(const float* steps, int ns, BruteState* stt, const float* bsad, const int* bidx,
                             int nblk, int n, int check, int scale) {
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (f >= n) return;
  BruteState s = stt[f];
  if (s.status != 0) return;
  float best = INFINITY;
  int bi = -1;
  for (int b = lane; b < nblk; b += 64) {
    const float sb = bsad[(size_t)f * nblk + b];
    const int ib = bidx[(size_t)f * nblk + b];
    if (brute_better(sb, ib, best, bi)) {
      best = sb;
      bi = ib;
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const float os = __shfl_xor(best, m);
    const int oi = __shfl_xor(bi, m);
    if (brute_better(os, oi, best, bi)) {
      best = os;
      bi = oi;
    }
  }
  if (lane != 0) return;
  float sel = 1e6f;
  if (bi >= 0 && !(best > 1e6f)) {
    s.x = s.x + steps[bi / ns];
    s.y = s.y + steps[bi % ns];
    sel = best;
  }
  s.sad = sel;
  if (check && sel > 100) s.status = 2;
  else if (scale) {
    s.x = (float)(s.x * 2.);
    s.y = (float)(s.y * 2.);
  }
  stt[f] = s;
}

std::vector<float> GaussianKernel5(double sigma) {   // getGaussianKernel(5, sigma, CV_32F)
  std::vector<float> k(5);
  const double scale2X = -0.5 / (sigma * sigma);
  double sum = 0.0;
  for (int i = 0; i < 5; ++i) {
    const double x = i - 2.0;
    k[i] = (float)std::exp(scale2X * x * x);
    sum += k[i];
  }
  sum = 1.0 / sum;
  for (int i = 0; i < 5; ++i) k[i] = (float)(k[i] * sum);
  return k;
}

Blur5 MakeBlur(double sigma) {
  const std::vector<float> k = GaussianKernel5(sigma);
  return Blur5{k[2], k[3], k[4]};
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// Host side

Tracker::Tracker(const sg_tracker_options& o, const sg_device_options& d) : opt_(o), dev_(d) {
  SG_REQUIRE(o.window >= 1 && o.window <= 16, SG_EINVAL, "window must be 1..16");
  SG_REQUIRE(o.depth >= 1 && o.depth <= kTrkMaxDepth, SG_EINVAL, "depth must be 1..8");
  SG_REQUIRE(o.max_images >= 1 && o.max_images <= 64, SG_EINVAL, "max_images must be 1..64");
  SG_REQUIRE(o.max_iterations >= 0, SG_EINVAL, "bad max_iterations");
  SG_REQUIRE(o.mode >= SG_TRACKER_HESSIAN && o.mode <= SG_TRACKER_BRUTE, SG_EINVAL, "bad tracker mode");
  int ndev = 0;
  SG_HIP_CHECK(hipGetDeviceCount(&ndev));
  SG_REQUIRE(ndev > 0 && d.device >= 0 && d.device < ndev, SG_ENODEV, "no such HIP device");
  SG_HIP_CHECK(hipSetDevice(d.device));
  stamp_on_ = getenv("SG_TRK_STAMP") && getenv("SG_TRK_STAMP")[0] == '1';
  SG_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  SG_HIP_CHECK(hipEventCreate(&ev_[0]));
  SG_HIP_CHECK(hipEventCreate(&ev_[1]));
  SG_HIP_CHECK(hipEventCreate(&ev_[2]));
  SG_HIP_CHECK(hipEventCreate(&ev_[3]));
  slots_.resize(o.max_images);
  // hessian.h:11-30 mask
  const int W = o.window, len = W * W;
  std::vector<float> m(len);
  for (int y = 0; y < W; ++y)
    for (int x = 0; x < W; ++x) {
      const double rx = 0.5 * W - x, ry = 0.5 * W - y, rr = rx * rx + ry * ry;
      m[y * W + x] = (float)(1. / (15. + rr));
    }
  double sum = 0.0;
  for (float v : m) sum += v;
  const double scale = len / sum;
  for (float& v : m) v = (float)(v * scale);
  mask_.Upload(m, stream_);
}

Tracker::~Tracker() {
  (void)hipSetDevice(dev_.device);
  for (auto& e : ev_)
    if (e) (void)hipEventDestroy(e);
  if (stream_) (void)hipStreamDestroy(stream_);
}

void Tracker::SetImage(int slot, const uint8_t* bgr, int w, int h, int stride) {
  SG_REQUIRE(slot >= 0 && slot < (int)slots_.size(), SG_EINVAL, "bad slot");
  SG_REQUIRE(bgr && w > 0 && h > 0 && stride >= 3 * w, SG_EINVAL, "bad image");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  Slot& s = slots_[slot];
  s.w.assign(opt_.depth, 0);
  s.h.assign(opt_.depth, 0);
  s.off.assign(opt_.depth, 0);
  size_t total = 0;
  int cw = w, ch = h;
  for (int l = 0; l < opt_.depth; ++l) {
    s.w[l] = cw;
    s.h[l] = ch;
    s.off[l] = total;
    total += (size_t)cw * ch;
    cw = (cw + 1) / 2;
    ch = (ch + 1) / 2;
  }
  s.pyr.Resize(total);
  tmp_.Resize((size_t)w * h);
  tmp2_.Resize((size_t)w * h);
  img_.Resize((size_t)stride * h);
  SG_HIP_CHECK(hipMemcpyAsync(img_.ptr, bgr, (size_t)stride * h, hipMemcpyHostToDevice, stream_));
  // hessian.h:95-126: blur 1.1 at level 0, pyrDown + blur 0.8 per level; klt.h:100-130: no blur at level 0,
  // pyrDown + blur 0.6; brute.h:60-80: no blur at all
  const int mode = opt_.mode;
  const Blur5 b0 = MakeBlur(1.1), b1 = MakeBlur(mode == SG_TRACKER_KLT ? 0.6 : 0.8);
  SG_HIP_CHECK(hipEventRecord(ev_[2], stream_));
  const int bx = 256;
  if (mode == SG_TRACKER_HESSIAN) {
    hipLaunchKernelGGL(k_gray_blur_row, dim3((w + bx - 1) / bx, h), dim3(bx), 0, stream_, img_.ptr, w, h, stride, b0,
                       tmp_.ptr);
    hipLaunchKernelGGL(k_blur_col, dim3((w + bx - 1) / bx, h), dim3(bx), 0, stream_, tmp_.ptr, w, h, b0, s.pyr.ptr);
  } else {
    hipLaunchKernelGGL(k_gray_scale, dim3((w + bx - 1) / bx, h), dim3(bx), 0, stream_, img_.ptr, w, h, stride,
                       s.pyr.ptr);
  }
  for (int l = 1; l < opt_.depth; ++l) {
    const int pw = s.w[l - 1], ph = s.h[l - 1], ow = s.w[l], oh = s.h[l];
    const bool blur = mode != SG_TRACKER_BRUTE;
    hipLaunchKernelGGL(k_pyrdown, dim3((ow + bx - 1) / bx, oh), dim3(bx), 0, stream_, s.pyr.ptr + s.off[l - 1], pw,
                       ph, blur ? tmp_.ptr : s.pyr.ptr + s.off[l], ow, oh);
    if (!blur) continue;
    hipLaunchKernelGGL(k_blur_row, dim3((ow + bx - 1) / bx, oh), dim3(bx), 0, stream_, tmp_.ptr, ow, oh, b1,
                       tmp2_.ptr);
    hipLaunchKernelGGL(k_blur_col, dim3((ow + bx - 1) / bx, oh), dim3(bx), 0, stream_, tmp2_.ptr, ow, oh, b1,
                       s.pyr.ptr + s.off[l]);
  }
  SG_HIP_CHECK(hipEventRecord(ev_[3], stream_));
  s.grey.Resize((size_t)w * h);
  hipLaunchKernelGGL(k_grey_u8, dim3((w + bx - 1) / bx, h), dim3(bx), 0, stream_, img_.ptr, w, h, stride, s.grey.ptr);
  SG_HIP_CHECK(hipGetLastError());
  // level table for the tracking kernel: {image, width, height} per level (scalar-loaded on the device)
  std::vector<uint8_t> tab(sizeof(LevelDev) * opt_.depth);
  for (int l = 0; l < opt_.depth; ++l) {
    LevelDev L{s.pyr.ptr + s.off[l], s.w[l], s.h[l]};
    std::memcpy(tab.data() + sizeof(LevelDev) * l, &L, sizeof(L));
  }
  s.table.Upload(tab, stream_);
  tabs_h_.resize(sizeof(LevelDev) * kTrkMaxDepth * slots_.size());
  std::memcpy(tabs_h_.data() + sizeof(LevelDev) * kTrkMaxDepth * slot, tab.data(), tab.size());
  tabs_.Upload(tabs_h_, stream_);
  SG_HIP_CHECK(hipStreamSynchronize(stream_));   // the host image buffer may be reused by the caller
  float ms = 0.f;
  SG_HIP_CHECK(hipEventElapsedTime(&ms, ev_[2], ev_[3]));
  pyr_ms_ = ms;
  s.valid = true;
}

void Tracker::GetLevel(int slot, int level, float* out, int* w, int* h) {
  SG_REQUIRE(slot >= 0 && slot < (int)slots_.size() && slots_[slot].valid, SG_EINVAL, "empty slot");
  SG_REQUIRE(level >= 0 && level < opt_.depth, SG_EINVAL, "bad level");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  const Slot& s = slots_[slot];
  *w = s.w[level];
  *h = s.h[level];
  if (out)
    SG_HIP_CHECK(hipMemcpyAsync(out, s.pyr.ptr + s.off[level], sizeof(float) * s.w[level] * s.h[level],
                                hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
}

void Tracker::GetPatches(int slot, int level, int n, const float* xy, float* out, float* mean, float* sumsq) {
  SG_REQUIRE(slot >= 0 && slot < (int)slots_.size() && slots_[slot].valid, SG_EINVAL, "empty slot");
  SG_REQUIRE(level >= 0 && level < opt_.depth && n >= 0, SG_EINVAL, "bad level / count");
  if (n == 0) return;
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  const Slot& s = slots_[slot];
  const int len = opt_.window * opt_.window;
  DBuf<float> dxy, dout, dm, dq;
  dxy.Upload(std::vector<float>(xy, xy + 2 * n), stream_);
  dout.Resize((size_t)n * len);
  dm.Resize(n);
  dq.Resize(n);
  LevelDev L{s.pyr.ptr + s.off[level], s.w[level], s.h[level]};
  hipLaunchKernelGGL(k_get_patches, dim3((n + kTrackWaves - 1) / kTrackWaves), dim3(64 * kTrackWaves), 0, stream_, L,
                     opt_.window, n, dxy.ptr, dout.ptr, dm.ptr, dq.ptr);
  SG_HIP_CHECK(hipGetLastError());
  SG_HIP_CHECK(hipMemcpyAsync(out, dout.ptr, sizeof(float) * n * len, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipMemcpyAsync(mean, dm.ptr, sizeof(float) * n, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipMemcpyAsync(sumsq, dq.ptr, sizeof(float) * n, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
}

void Tracker::LoadFeatures(int n, const float* from_xy, const float* to_xy, const int32_t* levels) {
  SG_REQUIRE(n >= 0 && (n == 0 || (from_xy && to_xy)), SG_EINVAL, "bad features");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  n_ = n;
  from_.Upload(std::vector<float>(from_xy, from_xy + 2 * (size_t)n), stream_);
  init_.Upload(std::vector<float>(to_xy, to_xy + 2 * (size_t)n), stream_);
  std::vector<int32_t> lv(n, 3);
  if (levels)
    for (int i = 0; i < n; ++i) lv[i] = levels[i];
  for (int v : lv) SG_REQUIRE(v >= 1, SG_EINVAL, "levels must be >= 1");
  levels_.Upload(lv, stream_);
  out_.Resize(2 * (size_t)std::max(n, 1));
  acc_.Resize(std::max(n, 1));
  its_.Resize(std::max(n, 1));
}

// Launch KERN<NK> for a W x W window (NK = ceil(W^2 / 64) patch pixels per lane, W <= 16).
#define SG_TRK_NK(W, KERN, ...)                                              \
  switch (((W) * (W) + 63) / 64) {                                           \
    case 1: hipLaunchKernelGGL(KERN<1>, __VA_ARGS__); break;                 \
    case 2: hipLaunchKernelGGL(KERN<2>, __VA_ARGS__); break;                 \
    case 3: hipLaunchKernelGGL(KERN<3>, __VA_ARGS__); break;                 \
    default: hipLaunchKernelGGL(KERN<4>, __VA_ARGS__); break;                \
  }

void Tracker::Run(int from, int to, int repeats) {
  SG_REQUIRE(from >= 0 && from < (int)slots_.size() && slots_[from].valid, SG_EINVAL, "empty 'from' slot");
  SG_REQUIRE(to >= 0 && to < (int)slots_.size() && slots_[to].valid, SG_EINVAL, "empty 'to' slot");
  SG_REQUIRE(repeats >= 1, SG_EINVAL, "repeats must be >= 1");
  const Slot& a = slots_[from];
  const Slot& b = slots_[to];
  SG_REQUIRE(a.w == b.w && a.h == b.h, SG_EINVAL, "pyramids of different sizes");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  TrackParams prm{opt_.window, opt_.max_iterations, opt_.threshold, opt_.fb_max, opt_.retry_levels, mask_.ptr};
  if (stamp_on_) {
    if (stamps_.size == 0) {
      stamps_.Resize(kTrkStamps);
      stamps_.Zero(stream_);
    }
    prm.stamps = stamps_.ptr;
  }
  SG_HIP_CHECK(hipEventRecord(ev_[0], stream_));
  if (n_ > 0)
    for (int r = 0; r < repeats; ++r)
      SG_TRK_NK(opt_.window, k_track_fb, dim3((n_ + kTrackWaves - 1) / kTrackWaves), dim3(64 * kTrackWaves), 0,
                stream_, (const LevelDev*)a.table.ptr, (const LevelDev*)b.table.ptr, opt_.depth, prm, n_, from_.ptr,
                init_.ptr, levels_.ptr, out_.ptr, acc_.ptr, its_.ptr);
  SG_HIP_CHECK(hipEventRecord(ev_[1], stream_));
  SG_HIP_CHECK(hipGetLastError());
  ran_ = true;
}

void Tracker::FindMatches(int to, int n, const int32_t* aoff, const int32_t* aslot, const float* axy,
                          const int32_t* levels, float* to_xy, int32_t* which, int32_t* iterations) {
  SG_REQUIRE(to >= 0 && to < (int)slots_.size() && slots_[to].valid, SG_EINVAL, "empty 'to' slot");
  SG_REQUIRE(n >= 0, SG_EINVAL, "bad feature count");
  if (n == 0) return;
  SG_REQUIRE(aoff && levels && to_xy && which && aoff[0] == 0, SG_EINVAL, "bad attempt lists");
  const int na = aoff[n];
  for (int f = 0; f < n; ++f) SG_REQUIRE(aoff[f + 1] >= aoff[f] && levels[f] >= 1, SG_EINVAL, "bad attempt lists");
  for (int a = 0; a < na; ++a) {
    SG_REQUIRE(aslot[a] >= 0 && aslot[a] < (int)slots_.size() && slots_[aslot[a]].valid, SG_EINVAL,
               "attempt from an empty slot");
    SG_REQUIRE(slots_[aslot[a]].w == slots_[to].w && slots_[aslot[a]].h == slots_[to].h, SG_EINVAL,
               "pyramids of different sizes");
  }
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  aoff_.Upload(std::vector<int32_t>(aoff, aoff + n + 1), stream_);
  aslot_.Upload(std::vector<int32_t>(aslot, aslot + std::max(na, 1)), stream_);
  axy_.Upload(std::vector<float>(axy, axy + 4 * (size_t)std::max(na, 1)), stream_);
  levels_.Upload(std::vector<int32_t>(levels, levels + n), stream_);
  out_.Resize(2 * (size_t)n);
  acc_.Resize(n);
  its_.Resize(n);
  TrackParams prm{opt_.window, opt_.max_iterations, opt_.threshold, opt_.fb_max, opt_.retry_levels, mask_.ptr};
  SG_HIP_CHECK(hipEventRecord(ev_[0], stream_));
  SG_TRK_NK(opt_.window, k_find_matches, dim3((n + kTrackWaves - 1) / kTrackWaves), dim3(64 * kTrackWaves), 0,
            stream_, (const LevelDev*)tabs_.ptr, to, opt_.depth, prm, n, aoff_.ptr, aslot_.ptr,
            reinterpret_cast<const float4*>(axy_.ptr), levels_.ptr, out_.ptr, acc_.ptr, its_.ptr);
  SG_HIP_CHECK(hipEventRecord(ev_[1], stream_));
  SG_HIP_CHECK(hipGetLastError());
  SG_HIP_CHECK(hipMemcpyAsync(to_xy, out_.ptr, sizeof(float) * 2 * n, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipMemcpyAsync(which, acc_.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, stream_));
  if (iterations)
    SG_HIP_CHECK(hipMemcpyAsync(iterations, its_.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
  float ms = 0.f;
  SG_HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
  track_ms_ = ms;
  ran_ = false;   // the batch buffers now hold this call's lists, not a LoadFeatures batch
  n_ = 0;
}

std::vector<unsigned long long> Tracker::Stamps() {
  std::vector<unsigned long long> v(kTrkStamps, 0);
  if (!stamp_on_ || stamps_.size == 0) return v;
  SG_HIP_CHECK(hipMemcpyAsync(v.data(), stamps_.ptr, kTrkStamps * 8, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
  stamps_.Zero(stream_);
  return v;
}

void Tracker::Results(float* to_xy, int32_t* accepted, int32_t* iterations) {
  SG_REQUIRE(ran_, SG_EINVAL, "no tracking run");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  if (n_ > 0) {
    if (to_xy) SG_HIP_CHECK(hipMemcpyAsync(to_xy, out_.ptr, sizeof(float) * 2 * n_, hipMemcpyDeviceToHost, stream_));
    if (accepted)
      SG_HIP_CHECK(hipMemcpyAsync(accepted, acc_.ptr, sizeof(int32_t) * n_, hipMemcpyDeviceToHost, stream_));
    if (iterations)
      SG_HIP_CHECK(hipMemcpyAsync(iterations, its_.ptr, sizeof(int32_t) * n_, hipMemcpyDeviceToHost, stream_));
  }
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
  float ms = 0.f;
  SG_HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
  track_ms_ = ms;
}

// One-directional TrackFeature of the configured FeatureTracker for n features (sg_tracker_track_feature).
void Tracker::TrackFeature(int from, int to, int n, const float* from_xy, float* to_xy, const int32_t* levels,
                           int32_t* status, int32_t* iterations) {
  SG_REQUIRE(from >= 0 && from < (int)slots_.size() && slots_[from].valid, SG_EINVAL, "empty 'from' slot");
  SG_REQUIRE(to >= 0 && to < (int)slots_.size() && slots_[to].valid, SG_EINVAL, "empty 'to' slot");
  SG_REQUIRE(n >= 0 && (n == 0 || (from_xy && to_xy && status)), SG_EINVAL, "bad features");
  const Slot& a = slots_[from];
  const Slot& b = slots_[to];
  SG_REQUIRE(a.w == b.w && a.h == b.h, SG_EINVAL, "pyramids of different sizes");
  if (n == 0) return;
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  hipStream_t st = stream_;
  const int depth = opt_.depth, W = opt_.window;
  from_.Upload(std::vector<float>(from_xy, from_xy + 2 * (size_t)n), st);
  out_.Upload(std::vector<float>(to_xy, to_xy + 2 * (size_t)n), st);
  if (levels) {
    for (int i = 0; i < n; ++i) SG_REQUIRE(levels[i] >= 1, SG_EINVAL, "levels must be >= 1");
    levels_.Upload(std::vector<int32_t>(levels, levels + n), st);
  }
  acc_.Resize(n);
  its_.Resize(n);
  its_.Zero(st);
  TrackParams prm{W, opt_.max_iterations, opt_.threshold, opt_.fb_max, opt_.retry_levels, mask_.ptr};
  const LevelDev* la = (const LevelDev*)a.table.ptr;
  const LevelDev* lb = (const LevelDev*)b.table.ptr;
  const dim3 grid((n + kTrackWaves - 1) / kTrackWaves), block(64 * kTrackWaves);
  if (opt_.mode == SG_TRACKER_HESSIAN) {
    SG_TRK_NK(W, k_track_one, grid, block, 0, st, la, lb, depth, prm, n, from_.ptr, out_.ptr,
              levels ? (const int32_t*)levels_.ptr : nullptr, acc_.ptr, its_.ptr);
  } else if (opt_.mode == SG_TRACKER_KLT) {
    hipLaunchKernelGGL(k_track_klt, grid, block, 0, st, la, lb, depth, prm, n, from_.ptr, out_.ptr, acc_.ptr,
                       its_.ptr);
  } else {
    SG_REQUIRE(n <= 65535, SG_EINVAL, "at most 65535 features per brute-force call");
    // brute.h:129-164: two passes per coarse level, five at level 0, each an exhaustive SearchBest grid
    struct Pass {
      float window, res;
      int lvl, check, scale;
    };
    std::vector<Pass> passes;
    for (int l = depth - 1; l > 0; --l) {
      passes.push_back({3.f, 1.f, l, 0, 0});
      passes.push_back({1.f, 0.33333f, l, 1, 1});
    }
    passes.push_back({3.f, 1.f, 0, 0, 0});
    passes.push_back({1.f, 0.3333f, 0, 0, 0});
    passes.push_back({0.4f, 0.1f, 0, 0, 0});
    passes.push_back({0.2f, 0.025f, 0, 0, 0});
    passes.push_back({8.f, 0.01f, 0, 1, 0});
    std::vector<float> steps;
    std::vector<int> soff, sn;
    int max_nblk = 1;
    for (const Pass& p : passes) {
      soff.push_back((int)steps.size());
      int cnt = 0;
      for (float x = -p.window; x <= p.window; x += p.res) {   // the reference's float stepping
        steps.push_back(x);
        ++cnt;
      }
      sn.push_back(cnt);
      max_nblk = std::max(max_nblk, (cnt * cnt + kBruteThreads - 1) / kBruteThreads);
    }
    brute_steps_.Upload(steps, st);
    brute_tmpl_.Resize((size_t)n * depth * (W * W + 2));
    brute_state_.Resize(sizeof(BruteState) * (size_t)n);
    brute_sad_.Resize((size_t)n * max_nblk);
    brute_idx_.Resize((size_t)n * max_nblk);
    BruteState* stt = reinterpret_cast<BruteState*>(brute_state_.ptr);
    hipLaunchKernelGGL(k_brute_setup, dim3((n * depth + 255) / 256), dim3(256), 0, st, la, lb, depth, W, n,
                       from_.ptr, out_.ptr, brute_tmpl_.ptr, stt);
    for (size_t k = 0; k < passes.size(); ++k) {
      const int ns = sn[k], nblk = (ns * ns + kBruteThreads - 1) / kBruteThreads;
      hipLaunchKernelGGL(k_brute_eval, dim3(nblk, n), dim3(kBruteThreads), 0, st, lb, passes[k].lvl, W, depth,
                         brute_tmpl_.ptr, brute_steps_.ptr + soff[k], ns, stt, brute_sad_.ptr, brute_idx_.ptr, nblk);
      hipLaunchKernelGGL(k_brute_pick, dim3((n + 3) / 4), dim3(256), 0, st, brute_steps_.ptr + soff[k], ns, stt,
                         brute_sad_.ptr, brute_idx_.ptr, nblk, n, passes[k].check, passes[k].scale);
    }
    SG_HIP_CHECK(hipGetLastError());
    std::vector<BruteState> hs(n);
    SG_HIP_CHECK(hipMemcpyAsync(hs.data(), stt, sizeof(BruteState) * (size_t)n, hipMemcpyDeviceToHost, st));
    SG_HIP_CHECK(hipStreamSynchronize(st));
    for (int i = 0; i < n; ++i) {
      status[i] = hs[i].status;
      if (hs[i].status == 0) {
        to_xy[2 * i] = hs[i].x;
        to_xy[2 * i + 1] = hs[i].y;
      }
      if (iterations) iterations[i] = 0;
    }
    return;
  }
  SG_HIP_CHECK(hipGetLastError());
  SG_HIP_CHECK(hipMemcpyAsync(to_xy, out_.ptr, sizeof(float) * 2 * (size_t)n, hipMemcpyDeviceToHost, st));
  SG_HIP_CHECK(hipMemcpyAsync(status, acc_.ptr, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, st));
  if (iterations)
    SG_HIP_CHECK(hipMemcpyAsync(iterations, its_.ptr, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, st));
  SG_HIP_CHECK(hipStreamSynchronize(st));
}

}  // namespace sg

