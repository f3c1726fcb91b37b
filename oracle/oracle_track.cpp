// oracle_track.cpp — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's front end (the
// HessianTracker of hessian.h and the forward/backward matcher of matcher.cpp), used by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker of the device tracker.
//
// The reference delegates image primitives to OpenCV 2.x (unpinned system library, not vendored and not
// installed here).  Their published algorithms are restated below (OpenCV 2.4 imgproc: color.cpp
// RGB2Gray<uchar>, convert.cpp cvtScale_, smooth.cpp getGaussianKernel + separable filter with
// BORDER_REFLECT_101, pyramids.cpp pyrDown_, samplers.cpp getRectSubPix_Cn_ + adjustRect).  Parity is
// unpinned by the reference (no fixtures for this path; OpenCV unavailable): see DESIGN.md.
// Arithmetic is float in the textbook left-to-right order (compiled with -ffp-contract=off); the
// reference's -ffast-math build may reassociate, so device/oracle tolerances are stated in the tests.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace oracle_trk {

// ------------------------------------------------------------------------------------------------
// OpenCV primitives (restated)

inline int Reflect101(int p, int n) {   // borderInterpolate(p, n, BORDER_REFLECT_101)
  if (n == 1) return 0;
  while (p < 0 || p >= n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
  }
  return p;
}

// cvtColor(img, grey, CV_RGB2GRAY) on an 8UC3 image whose memory order is BGR (hessian.h:100): the
// weights meant for R are applied to channel 0.  Fixed point, yuv_shift 14.
void RgbToGrayU8(const uint8_t* src, int w, int h, int stride, uint8_t* dst) {
  const int R2Y = 4899, G2Y = 9617, B2Y = 1868, shift = 14;
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const uint8_t* p = src + (size_t)y * stride + 3 * x;
      dst[(size_t)y * w + x] = (uint8_t)((R2Y * p[0] + G2Y * p[1] + B2Y * p[2] + (1 << (shift - 1))) >> shift);
    }
}

// getGaussianKernel(n, sigma, CV_32F) for sigma > 0.
std::vector<float> GaussianKernel(int n, double sigma) {
  std::vector<float> k(n);
  const double scale2X = -0.5 / (sigma * sigma);
  double sum = 0.0;
  for (int i = 0; i < n; ++i) {
    const double x = i - (n - 1) * 0.5;
    k[i] = (float)std::exp(scale2X * x * x);
    sum += k[i];
  }
  sum = 1.0 / sum;
  for (int i = 0; i < n; ++i) k[i] = (float)(k[i] * sum);
  return k;
}

// GaussianBlur(img, img, Size(5,5), sigma, sigma): separable symmetric 5-tap, rows then columns,
// BORDER_REFLECT_101; s = c*k0 + (l1 + r1)*k1 + (l2 + r2)*k2.
void GaussianBlur5(std::vector<float>& img, int w, int h, double sigma) {
  const std::vector<float> k = GaussianKernel(5, sigma);
  const float k0 = k[2], k1 = k[3], k2 = k[4];
  std::vector<float> tmp((size_t)w * h);
  for (int y = 0; y < h; ++y) {
    const float* r = &img[(size_t)y * w];
    for (int x = 0; x < w; ++x) {
      const float c = r[x];
      const float l1 = r[Reflect101(x - 1, w)], r1 = r[Reflect101(x + 1, w)];
      const float l2 = r[Reflect101(x - 2, w)], r2 = r[Reflect101(x + 2, w)];
      tmp[(size_t)y * w + x] = c * k0 + (l1 + r1) * k1 + (l2 + r2) * k2;
    }
  }
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const float c = tmp[(size_t)y * w + x];
      const float u1 = tmp[(size_t)Reflect101(y - 1, h) * w + x], d1 = tmp[(size_t)Reflect101(y + 1, h) * w + x];
      const float u2 = tmp[(size_t)Reflect101(y - 2, h) * w + x], d2 = tmp[(size_t)Reflect101(y + 2, h) * w + x];
      img[(size_t)y * w + x] = c * k0 + (u1 + d1) * k1 + (u2 + d2) * k2;
    }
}

// pyrDown(src, dst): 1-4-6-4-1 rows then columns, BORDER_REFLECT_101, scale 1/256, dst ((w+1)/2, (h+1)/2).
void PyrDown(const std::vector<float>& src, int w, int h, std::vector<float>& dst, int* dw, int* dh) {
  const int ow = (w + 1) / 2, oh = (h + 1) / 2;
  std::vector<float> rows((size_t)ow * h);
  for (int y = 0; y < h; ++y) {
    const float* s = &src[(size_t)y * w];
    for (int x = 0; x < ow; ++x) {
      const int c = 2 * x;
      rows[(size_t)y * ow + x] = s[Reflect101(c, w)] * 6 + (s[Reflect101(c - 1, w)] + s[Reflect101(c + 1, w)]) * 4 +
                                 s[Reflect101(c - 2, w)] + s[Reflect101(c + 2, w)];
    }
  }
  dst.assign((size_t)ow * oh, 0.f);
  for (int y = 0; y < oh; ++y) {
    const int c = 2 * y;
    const float* r0 = &rows[(size_t)Reflect101(c - 2, h) * ow];
    const float* r1 = &rows[(size_t)Reflect101(c - 1, h) * ow];
    const float* r2 = &rows[(size_t)Reflect101(c, h) * ow];
    const float* r3 = &rows[(size_t)Reflect101(c + 1, h) * ow];
    const float* r4 = &rows[(size_t)Reflect101(c + 2, h) * ow];
    for (int x = 0; x < ow; ++x)
      dst[(size_t)y * ow + x] = (r2[x] * 6 + (r1[x] + r3[x]) * 4 + r0[x] + r4[x]) * (1.f / 256.f);
  }
  *dw = ow;
  *dh = oh;
}

// getRectSubPix(src, Size(pw, ph), center, dst) for CV_32F -> CV_32F (getRectSubPix_Cn_ with adjustRect:
// bilinear inside, replicated border outside).
void GetRectSubPix(const float* img, int w, int h, int pw, int ph, float cx, float cy, float* dst, int dstride) {
  cx -= (pw - 1) * 0.5f;
  cy -= (ph - 1) * 0.5f;
  const int ipx = (int)std::floor(cx), ipy = (int)std::floor(cy);
  const float a = cx - ipx, b = cy - ipy;
  const float a11 = (1.f - a) * (1.f - b), a12 = a * (1.f - b), a21 = (1.f - a) * b, a22 = a * b;
  const float b1 = 1.f - b, b2 = b;
  // adjustRect
  int base_col, base_row, rx, rw, ry, rh;
  if (ipx >= 0) { base_col = ipx; rx = 0; }
  else { base_col = 0; rx = std::min(-ipx, pw); }
  if (ipx < w - pw) rw = pw;
  else {
    rw = w - ipx - 1;
    if (rw < 0) { base_col += rw; rw = 0; }
  }
  if (ipy >= 0) { base_row = ipy; ry = 0; }
  else { base_row = 0; ry = -ipy; }
  if (ipy < h - ph) rh = ph;
  else {
    rh = h - ipy - 1;
    if (rh < 0) { base_row += rh; rh = 0; }
  }
  const int col0 = base_col - rx;   // src pointer column after "src - rect.x"
  int row = base_row;
  for (int i = 0; i < ph; ++i) {
    const bool same = (i < ry || i >= rh);
    const float* s1 = img + (size_t)row * w;
    const float* s2 = same ? s1 : s1 + w;
    float* d = dst + (size_t)i * dstride;
    int j = 0;
    for (; j < rx; ++j) d[j] = s1[col0 + rx] * b1 + s2[col0 + rx] * b2;
    for (; j < rw; ++j) d[j] = s1[col0 + j] * a11 + s1[col0 + j + 1] * a12 + s2[col0 + j] * a21 + s2[col0 + j + 1] * a22;
    for (; j < pw; ++j) d[j] = s1[col0 + rw] * b1 + s2[col0 + rw] * b2;
    if (i < rh && !same) ++row;
  }
}

// ------------------------------------------------------------------------------------------------
// HessianTracker (hessian.h)

struct Patch {
  std::vector<float> data;
  float mean = 0.f, sumsq = 0.f;
};

// Fixed summation order for the patch sums (the reference sums sequentially in a -ffast-math build, i.e.
// in a compiler-chosen vectorised order): 64 lane partials, partial[l] = sum over i = l (mod 64) in
// increasing i, then a pairwise tree over consecutive partials.  This is the order of the device
// tracker (one wave per track, DPP reduction), so the two agree bit for bit.
// 0: the lane-tree order below (the device's); 1: the reference's textbook loop order, left to right
// (hessian.h:86-88, 133-139 as written; its -ffast-math build may reassociate further).  Switchable so a
// test can measure how far the two orders move a track (1e-3 px).
static int g_sum_order = 0;

inline float LaneTreeSum(const float* v, int n) {
  if (g_sum_order == 1) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += v[i];
    return s;
  }
  float part[64];
  for (int l = 0; l < 64; ++l) part[l] = 0.f;
  for (int i = 0; i < n; ++i) part[i & 63] += v[i];
  for (int width = 64; width > 4; width >>= 1)
    for (int l = 0; l < width / 2; ++l) part[l] = part[2 * l] + part[2 * l + 1];
  return (part[0] + part[1]) + (part[2] + part[3]);
}

struct Tracker {
  int W, len;
  std::vector<float> mask;

  explicit Tracker(int win) : W(win), len(win * win), mask(win * win) {   // hessian.h:11-30
    for (int y = 0; y < W; ++y)
      for (int x = 0; x < W; ++x) {
        const double rx = 0.5 * W - x, ry = 0.5 * W - y, rr = rx * rx + ry * ry;
        mask[y * W + x] = (float)(1. / (15. + rr));
      }
    double sum = 0.0;
    for (float v : mask) sum += v;
    const double scale = len / sum;
    for (float& v : mask) v = (float)(v * scale);
  }

  // hessian.h:54-93: zero-filled left/top columns when the point is near the edge, then getRectSubPix.
  Patch GetPatch(const float* img, int w, int h, float px, float py) const {
    Patch p;
    p.data.assign(len, 0.f);
    int rx = 0, ry = 0, rw = W, rh = W;
    if (px < 0.5 * W) {
      const int d = (int)((0.5 * W - px) + 0.9999);
      px = (float)(px + 0.5 * d);
      rx = d;
      rw = W - d;
    }
    if (py < 0.5 * W) {
      const int d = (int)(0.5 * W - py);
      py = (float)(py + 0.5 * d);
      ry = d;
      rh = W - d;
    }
    if (rw > 0 && rh > 0) GetRectSubPix(img, w, h, rw, rh, px, py, &p.data[rx + ry * W], W);
    std::vector<float> sq(len);
    for (int i = 0; i < len; ++i) sq[i] = p.data[i] * p.data[i];
    const float sum = LaneTreeSum(p.data.data(), len), sum_sq = LaneTreeSum(sq.data(), len);
    p.mean = sum / len;
    p.sumsq = sum_sq / len;
    return p;
  }

  float Score(const Patch& p1, const Patch& p2) const {   // hessian.h:129-141
    const float alpha = std::sqrt(p1.sumsq / p2.sumsq);
    const float beta = p1.mean - alpha * p2.mean;
    std::vector<float> term(len, 0.f);
    for (int i = 0; i < len; ++i) {
      if (p1.data[i] == 0 || p2.data[i] == 0) continue;
      float diff = p1.data[i] - p2.data[i] * alpha - beta;
      diff = diff * diff;
      term[i] = diff * mask[i];
    }
    return LaneTreeSum(term.data(), len);
  }

  // hessian.h:147-172
  float BruteHessian(const float* img, int w, int h, const Patch& patch, float x, float y, float* dx, float* dy,
                     float* dxx, float* dxy, float* dyx, float* dyy) const {
    const double hh = 0.02;
    const double sad0 = Score(patch, GetPatch(img, w, h, x, y));
    const double sadn1x = Score(patch, GetPatch(img, w, h, (float)(x - hh), y));
    const double sadn1y = Score(patch, GetPatch(img, w, h, x, (float)(y - hh)));
    const double sadp1x = Score(patch, GetPatch(img, w, h, (float)(x + hh), y));
    const double sadp1y = Score(patch, GetPatch(img, w, h, x, (float)(y + hh)));
    const double sadxy = Score(patch, GetPatch(img, w, h, (float)(x + hh), (float)(y + hh)));
    *dx = (float)(0.5 * (sadp1x - sadn1x) / hh);
    *dy = (float)(0.5 * (sadp1y - sadn1y) / hh);
    *dxx = (float)(((sadp1x - sad0) / hh - (sad0 - sadn1x) / hh) / hh);
    *dyy = (float)(((sadp1y - sad0) / hh - (sad0 - sadn1y) / hh) / hh);
    *dxy = (float)(((sadxy - sadp1y) / hh - (sadp1x - sad0) / hh) / hh);
    *dyx = (float)(((sadxy - sadp1x) / hh - (sadp1y - sad0) / hh) / hh);
    return (float)sad0;
  }

  // hessian.h:185-241.  Returns 0 OK, 2 OUT_OF_BOUNDS; *iters = Newton iterations run.
  int Track(const float* img, int w, int h, const Patch& patch, float threshold, int max_iterations, float* px,
            float* py, int* iters) const {
    float x = *px, y = *py;
    const float margin = 0.01f;
    int it = 0;
    for (; it < max_iterations; ++it) {
      if (x < margin || y < margin || (x + margin) > w || (y + margin) > h) {
        *px = x;
        *py = y;
        if (iters) *iters += it;
        return 2;
      }
      float mdx, mdy, mdxx, mdxy, mdyx, mdyy;
      BruteHessian(img, w, h, patch, x, y, &mdx, &mdy, &mdxx, &mdxy, &mdyx, &mdyy);
      // Eigen Matrix2d inverse (cofactors / determinant) times g
      const double H00 = mdxx, H01 = mdxy, H10 = mdyx, H11 = mdyy;
      const double det = H00 * H11 - H10 * H01;
      const double invdet = 1.0 / det;
      const double i00 = H11 * invdet, i10 = -H10 * invdet, i01 = -H01 * invdet, i11 = H00 * invdet;
      const double g0 = mdx, g1 = mdy;
      const double jj0 = i00 * g0 + i01 * g1, jj1 = i10 * g0 + i11 * g1;
      float dx = (float)-jj0, dy = (float)-jj1;
      if ((dx * dx + dy * dy) > 1) {
        dx /= std::sqrt(dx * dx + dy * dy);
        dy /= std::sqrt(dx * dx + dy * dy);   // uses the updated dx (reference quirk)
      }
      // x += max(-1.f, min(1.f, dx)) with std::min/std::max NaN semantics
      const float cx = (dx < 1.f) ? dx : 1.f, cy = (dy < 1.f) ? dy : 1.f;
      x += (-1.f < cx) ? cx : -1.f;
      y += (-1.f < cy) ? cy : -1.f;
      if (std::fabs(dx) < threshold && std::fabs(dy) < threshold) {
        ++it;
        break;
      }
    }
    if (iters) *iters += it;
    *px = x;
    *py = y;
    return 0;
  }
};

struct Level {
  const float* img;
  int w, h;
};

// hessian.h:243-264 (TrackFeature) with GetPatches (175-183) for the source templates.
int TrackFeature(const Tracker& T, const std::vector<Level>& src, const std::vector<Level>& dst, float sx, float sy,
                 int levels, float threshold, int max_iterations, float* px, float* py, int* iters) {
  const int lvls = std::min((int)std::min(src.size(), dst.size()), levels);
  std::vector<Patch> patches(lvls);
  float tx = sx, ty = sy;
  for (int i = 0; i < lvls; ++i) {
    patches[i] = T.GetPatch(src[i].img, src[i].w, src[i].h, tx, ty);
    tx = (float)(tx * 0.5);
    ty = (float)(ty * 0.5);
  }
  const double s = 1. / (1 << (lvls - 1));
  float x = (float)(*px * s), y = (float)(*py * s);
  for (int i = lvls - 1; i > 0; --i) {
    const int st = T.Track(dst[i].img, dst[i].w, dst[i].h, patches[i], threshold, max_iterations, &x, &y, iters);
    if (st != 0) return st;
    x = (float)(x * 2.);
    y = (float)(y * 2.);
  }
  const int st = T.Track(dst[0].img, dst[0].w, dst[0].h, patches[0], threshold, max_iterations, &x, &y, iters);
  if (st != 0) return st;
  *px = x;
  *py = y;
  return 0;
}

// matcher.cpp:173-206 (forward/backward TrackFeature) and the 3 -> 6 level retry of matcher.cpp:247-251.
bool TrackFB(const Tracker& T, const std::vector<Level>& from, const std::vector<Level>& to, float fx, float fy,
             int levels, float* tx, float* ty, int* iters, int retry_levels = 6) {
  // The backward pass is skipped when the forward pass failed: the reference runs it but rejects the feature
  // either way (matcher.cpp:193), and it never modifies to_pt.  (Only the iteration count differs.)
  auto attempt = [&](int lv) {
    const int s1 = TrackFeature(T, from, to, fx, fy, lv, 0.001f, 10, tx, ty, iters);
    if (s1) return false;
    float bx = fx, by = fy;
    const int s2 = TrackFeature(T, to, from, *tx, *ty, lv, 0.001f, 10, &bx, &by, iters);
    if (s2) return false;
    const float ex = fx - bx, ey = fy - by;   // Point2f difference, then cv::norm in double
    return !(std::sqrt((double)ex * ex + (double)ey * ey) > 0.3);
  };
  if (attempt(levels)) return true;
  if (retry_levels <= 0 || levels == retry_levels) return false;   // sg_tracker_options.retry_levels
  return attempt(retry_levels);
}

}  // namespace oracle_trk

using namespace oracle_trk;

extern "C" {

void ort_set_sum_order(int order) { g_sum_order = order; }

// MakePyramid (hessian.h:95-126): BGR u8 -> grey -> /255 -> GaussianBlur(5, 1.1); then per level
// pyrDown + GaussianBlur(5, 0.8).  out holds the levels back to back; dims[2l], dims[2l+1] = w, h.
int ort_make_pyramid(const uint8_t* bgr, int w, int h, int stride, int depth, float* out, int32_t* dims) {
  std::vector<uint8_t> grey((size_t)w * h);
  RgbToGrayU8(bgr, w, h, stride, grey.data());
  std::vector<float> cur((size_t)w * h);
  const float sc = (float)(1. / 255.);
  for (size_t i = 0; i < cur.size(); ++i) cur[i] = (float)grey[i] * sc;
  GaussianBlur5(cur, w, h, 1.1);
  int cw = w, ch = h;
  size_t off = 0;
  for (int l = 0; l < depth; ++l) {
    if (l > 0) {
      std::vector<float> nxt;
      int nw, nh;
      PyrDown(cur, cw, ch, nxt, &nw, &nh);
      GaussianBlur5(nxt, nw, nh, 0.8);
      cur.swap(nxt);
      cw = nw;
      ch = nh;
    }
    std::memcpy(out + off, cur.data(), cur.size() * sizeof(float));
    dims[2 * l] = cw;
    dims[2 * l + 1] = ch;
    off += cur.size();
  }
  return 0;
}

int ort_get_rect_subpix(const float* img, int w, int h, int pw, int ph, float cx, float cy, float* out) {
  GetRectSubPix(img, w, h, pw, ph, cx, cy, out, pw);
  return 0;
}

int ort_get_patch(const float* img, int w, int h, int win, float x, float y, float* out, float* mean, float* sumsq) {
  Tracker T(win);
  Patch p = T.GetPatch(img, w, h, x, y);
  std::memcpy(out, p.data.data(), p.data.size() * sizeof(float));
  *mean = p.mean;
  *sumsq = p.sumsq;
  return 0;
}

int ort_mask(int win, float* out) {
  Tracker T(win);
  std::memcpy(out, T.mask.data(), T.mask.size() * sizeof(float));
  return 0;
}

// Forward/backward tracking of n features between two pyramids (same dims).  to_xy: in = initial guess,
// out = tracked position (as the matcher leaves it).  accepted[i] = FB check passed.  iters (optional):
// total Newton iterations per track.
int ort_track_fb(const float* pyr_from, const float* pyr_to, const int32_t* dims, int depth, int win, int n,
                 const float* from_xy, float* to_xy, const int32_t* levels, int32_t* accepted, int32_t* iters,
                 int nthreads, int retry_levels) {
  std::vector<Level> from(depth), to(depth);
  size_t off = 0;
  for (int l = 0; l < depth; ++l) {
    from[l] = Level{pyr_from + off, dims[2 * l], dims[2 * l + 1]};
    to[l] = Level{pyr_to + off, dims[2 * l], dims[2 * l + 1]};
    off += (size_t)dims[2 * l] * dims[2 * l + 1];
  }
  Tracker T(win);
#pragma omp parallel for schedule(dynamic, 8) num_threads(nthreads > 0 ? nthreads : 1)
  for (int i = 0; i < n; ++i) {
    int it = 0;
    accepted[i] = TrackFB(T, from, to, from_xy[2 * i], from_xy[2 * i + 1], levels ? levels[i] : 3, &to_xy[2 * i],
                          &to_xy[2 * i + 1], &it, retry_levels) ? 1 : 0;
    if (iters) iters[i] = it;
  }
  return 0;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// 256-bit descriptor all-pairs Hamming match (BASELINE config 4; SURVEY.md 8a row a19 — no reference
// implementation exists, the specification is: distance = popcount(a XOR b) over 4 x u64, per query the
// argmin over the train set with ties to the lowest train index, plus the second-smallest distance).
extern "C" int ort_hamming_match(const uint64_t* q, int nq, const uint64_t* t, int nt, int32_t* best_idx,
                                 int32_t* best_dist, int32_t* second_dist, int nthreads) {
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
  for (int i = 0; i < nq; ++i) {
    const uint64_t* a = q + 4 * (size_t)i;
    int bd = 1 << 30, sd = 1 << 30, bi = -1;
    for (int j = 0; j < nt; ++j) {
      const uint64_t* b = t + 4 * (size_t)j;
      const int d = __builtin_popcountll(a[0] ^ b[0]) + __builtin_popcountll(a[1] ^ b[1]) +
                    __builtin_popcountll(a[2] ^ b[2]) + __builtin_popcountll(a[3] ^ b[3]);
      if (d < bd) {
        sd = bd;
        bd = d;
        bi = j;
      } else if (d < sd) {
        sd = d;
      }
    }
    best_idx[i] = bi;
    best_dist[i] = nt > 0 ? bd : -1;
    second_dist[i] = nt > 1 ? sd : -1;
  }
  return 0;
}

// ------------------------------------------------------------------------------------------------
// Corner seeding of a new keyframe (matcher.cpp:123-169, AddNewFeatures): cvtColor(img, grey,
// CV_RGB2GRAY) (matcher.cpp:214) then goodFeaturesToTrack(grey, corners, 120, 0.01, 20) with OpenCV 2.4's
// defaults (blockSize 3, Shi-Tomasi), then the 30 x 30 grid suppression around the existing matches.
// OpenCV 2.4 imgproc restated: corner.cpp cornerEigenValsVecs / calcMinEigenVal (Sobel 3x3 scaled by
// 1 / (4 * 3 * 255) on the smoothing tap, boxFilter 3x3 unnormalised, BORDER_REFLECT_101), featureselect.cpp
// goodFeaturesToTrack (threshold at quality x max, 3x3 dilation = local maxima, strongest first, greedy
// minimum distance on a cell grid).  OpenCV sorts with std::sort (order of exactly equal responses
// implementation-defined); here ties go to the lower row-major index.  Float arithmetic in the order
// written (this file is compiled with -ffp-contract=off).
namespace oracle_trk {

// cornerMinEigenVal(grey, eig, 3, 3).
void MinEigen3(const uint8_t* g, int w, int h, float* eig) {
  const float s = (float)(1.0 / (4.0 * 3.0 * 255.0));
  const float k0 = 2.0f * s, k1 = s;   // scaled smoothing tap [s, 2s, s]
  std::vector<float> dx((size_t)w * h), dy((size_t)w * h);
  auto G = [&](int y, int x) { return (float)g[(size_t)Reflect101(y, h) * w + Reflect101(x, w)]; };
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float r[3], q[3];
      for (int k = 0; k < 3; ++k) {
        const int yy = y - 1 + k;
        r[k] = G(yy, x + 1) - G(yy, x - 1);                     // derivative row tap [-1, 0, 1]
        q[k] = G(yy, x) * k0 + (G(yy, x - 1) + G(yy, x + 1)) * k1;   // smoothing row tap
      }
      dx[(size_t)y * w + x] = r[1] * k0 + (r[0] + r[2]) * k1;   // smoothing column tap
      dy[(size_t)y * w + x] = q[2] - q[0];                      // derivative column tap
    }
  std::vector<float> c0((size_t)w * h), c1((size_t)w * h), c2((size_t)w * h);
  for (size_t i = 0; i < c0.size(); ++i) {
    c0[i] = dx[i] * dx[i];
    c1[i] = dx[i] * dy[i];
    c2[i] = dy[i] * dy[i];
  }
  auto box = [&](const std::vector<float>& c, int y, int x) {
    float col = 0.0f;
    for (int k = 0; k < 3; ++k) {
      const size_t row = (size_t)Reflect101(y - 1 + k, h) * w;
      const float rs = (c[row + Reflect101(x - 1, w)] + c[row + x]) + c[row + Reflect101(x + 1, w)];
      col = k == 0 ? rs : col + rs;
    }
    return col;
  };
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const float a = box(c0, y, x) * 0.5f, b = box(c1, y, x), c = box(c2, y, x) * 0.5f;
      eig[(size_t)y * w + x] = (a + c) - std::sqrt((a - c) * (a - c) + b * b);
    }
}

// goodFeaturesToTrack(grey, corners, max_corners, quality, min_distance) with its default mask / block
// size; corners as (x, y) pixel positions.
int GoodFeatures(const uint8_t* g, int w, int h, int max_corners, double quality, double min_distance,
                 std::vector<float>* corners) {
  std::vector<float> eig((size_t)w * h);
  MinEigen3(g, w, h, eig.data());
  float maxv = 0.0f;
  for (float v : eig) maxv = std::max(maxv, v);
  const float thr = (float)(maxv * quality);
  for (float& v : eig) v = v > thr ? v : 0.0f;   // THRESH_TOZERO
  std::vector<int> cand;
  for (int y = 1; y < h - 1; ++y)
    for (int x = 1; x < w - 1; ++x) {
      const float v = eig[(size_t)y * w + x];
      float m = v;
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) m = std::max(m, eig[(size_t)(y + dy) * w + x + dx]);
      if (v != 0 && v == m) cand.push_back(y * w + x);
    }
  std::stable_sort(cand.begin(), cand.end(), [&](int a, int b) { return eig[a] > eig[b]; });
  corners->clear();
  const int cell = (int)std::lround(min_distance);
  const int gw = (w + cell - 1) / cell, gh = (h + cell - 1) / cell;
  std::vector<std::vector<std::pair<float, float>>> grid((size_t)gw * gh);
  const double md2 = min_distance * min_distance;
  int n = 0;
  for (int idx : cand) {
    const int y = idx / w, x = idx % w;
    const int xc = x / cell, yc = y / cell;
    bool good = true;
    for (int yy = std::max(0, yc - 1); yy <= std::min(gh - 1, yc + 1) && good; ++yy)
      for (int xx = std::max(0, xc - 1); xx <= std::min(gw - 1, xc + 1) && good; ++xx)
        for (const auto& m : grid[(size_t)yy * gw + xx]) {
          const float ddx = x - m.first, ddy = y - m.second;
          if (ddx * ddx + ddy * ddy < md2) {
            good = false;
            break;
          }
        }
    if (!good) continue;
    grid[(size_t)yc * gw + xc].push_back({(float)x, (float)y});
    corners->push_back((float)x);
    corners->push_back((float)y);
    if (max_corners > 0 && ++n == max_corners) break;
  }
  return n;
}

// AddNewFeatures' cell of a point: (pt / size) * 30 + 1 in float, truncated (matcher.cpp:135-137).
inline int SeedCell(float v, int size) { return (int)(v / size * 30 + 1); }

}  // namespace oracle_trk

extern "C" {

// Matcher::Track's new-keyframe seeding: grey from the BGR frame, goodFeaturesToTrack(120, 0.01, 20), and
// AddNewFeatures' grid filter against the current matches.  corners_xy gets every corner (<= max_corners),
// added_xy the ones kept; returns the number kept (*num_corners = corners found).
int ort_seed_features(const uint8_t* bgr, int w, int h, int stride, const float* match_xy, int num_matches,
                      int max_corners, double quality, double min_distance, float* corners_xy, int32_t* num_corners,
                      float* added_xy) {
  using namespace oracle_trk;
  std::vector<uint8_t> grey((size_t)w * h);
  RgbToGrayU8(bgr, w, h, stride, grey.data());
  std::vector<float> corners;
  const int n = GoodFeatures(grey.data(), w, h, max_corners, quality, min_distance, &corners);
  *num_corners = n;
  std::copy(corners.begin(), corners.end(), corners_xy);
  int grid[32][32] = {};
  for (int i = 0; i < num_matches; ++i) {
    const int gx = SeedCell(match_xy[2 * i], w), gy = SeedCell(match_xy[2 * i + 1], h);
    if (gx <= 0 || gy <= 0 || gx >= 31 || gy >= 31) return -1;   // the reference CHECKs 0 < g < size + 2
    for (int a = -1; a <= 1; ++a)
      for (int b = -1; b <= 1; ++b) grid[gx + a][gy + b] = 1;
  }
  int added = 0;
  for (int i = 0; i < n; ++i) {
    const int gx = SeedCell(corners[2 * i], w), gy = SeedCell(corners[2 * i + 1], h);
    if (grid[gx][gy]) continue;
    added_xy[2 * added] = corners[2 * i];
    added_xy[2 * added + 1] = corners[2 * i + 1];
    ++added;
  }
  return added;
}

// cornerMinEigenVal(grey(bgr), eig, 3, 3) alone (checker of the device response image).
int ort_min_eigen(const uint8_t* bgr, int w, int h, int stride, float* eig) {
  std::vector<uint8_t> grey((size_t)w * h);
  oracle_trk::RgbToGrayU8(bgr, w, h, stride, grey.data());
  oracle_trk::MinEigen3(grey.data(), w, h, eig);
  return 0;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// The reference's two other FeatureTracker implementations.  Neither is
// executed by the reference (Matcher typedefs HessianTracker, matcher.cpp:20), so their restatements below
// are the specification of the device modes; they share the HessianTracker primitives above.
namespace oracle_trk {

// klt.h:105-135 / brute.h:60-80 MakePyramid: grey / 255, no blur at level 0; each further level pyrDown,
// then (klt.h only) GaussianBlur 5x5 sigma 0.6.  klt.h's Scharr gradient images (105-106, 119-125) feed only
// the LK matrices A, B, C, RS, VW of Track, whose result the reference overwrites with the BruteHessian
// step (klt.h:333-359): they do not influence any output and are not computed here.
void MakePyramidMode(int mode, const uint8_t* bgr, int w, int h, int stride, int depth, float* out, int32_t* dims) {
  std::vector<uint8_t> grey((size_t)w * h);
  RgbToGrayU8(bgr, w, h, stride, grey.data());
  std::vector<float> cur((size_t)w * h);
  const float sc = (float)(1. / 255.);
  for (size_t i = 0; i < cur.size(); ++i) cur[i] = (float)grey[i] * sc;
  int cw = w, ch = h;
  size_t off = 0;
  for (int l = 0; l < depth; ++l) {
    if (l > 0) {
      std::vector<float> nxt;
      int nw, nh;
      PyrDown(cur, cw, ch, nxt, &nw, &nh);
      if (mode == 1) GaussianBlur5(nxt, nw, nh, 0.6);
      cur.swap(nxt);
      cw = nw;
      ch = nh;
    }
    std::memcpy(out + off, cur.data(), cur.size() * sizeof(float));
    dims[2 * l] = cw;
    dims[2 * l + 1] = ch;
    off += cur.size();
  }
}

// klt.h / brute.h GetPatch: a plain W x W getRectSubPix (no edge shift).  `lane_sums` selects the patch-sum
// order: the KLT mode uses the one-wave-per-feature lane-tree order, the brute mode (one device thread per
// candidate) the sequential order of the reference's loop.
Patch PlainPatch(const Tracker& T, const float* img, int w, int h, float px, float py, bool lane_sums) {
  Patch p;
  p.data.assign(T.len, 0.f);
  GetRectSubPix(img, w, h, T.W, T.W, px, py, p.data.data(), T.W);
  float sum = 0.f, sum_sq = 0.f;
  if (lane_sums) {
    std::vector<float> sq(T.len);
    for (int i = 0; i < T.len; ++i) sq[i] = p.data[i] * p.data[i];
    sum = LaneTreeSum(p.data.data(), T.len);
    sum_sq = LaneTreeSum(sq.data(), T.len);
  } else {
    for (float d : p.data) {
      sum += d;
      sum_sq += d * d;
    }
  }
  p.mean = sum / T.len;
  p.sumsq = sum_sq / T.len;
  return p;
}

// klt.h:139-149 SADPatches(template, probe): masked, not lighting-normalised.
float KltScore(const Tracker& T, const Patch& p1, const Patch& p2) {
  std::vector<float> term(T.len, 0.f);
  for (int i = 0; i < T.len; ++i) {
    if (p1.data[i] == 0 || p2.data[i] == 0) continue;
    const float diff = p1.data[i] - p2.data[i];
    term[i] = diff * diff * T.mask[i];
  }
  return LaneTreeSum(term.data(), T.len);
}

// klt.h:258-401 Track with the BruteHessian of 181-204 (forward differences, h = 0.01); margin 0.1, stop when
// both steps are below threshold / 10.
int KltTrack(const Tracker& T, const Level& L, const Patch& patch, float threshold, int max_iterations, float* px,
             float* py, int* iters) {
  float x = *px, y = *py;
  const float margin = 0.1f;
  int it = 0;
  for (; it < max_iterations; ++it) {
    if (x < margin || y < margin || (x + margin) > L.w || (y + margin) > L.h) {
      if (iters) *iters += it;
      return 2;
    }
    const double hh = 0.01;
    auto S = [&](float qx, float qy) { return (double)KltScore(T, patch, PlainPatch(T, L.img, L.w, L.h, qx, qy, true)); };
    const double sad0 = S(x, y);
    const double sadx = S((float)(x + hh), y);
    const double sady = S(x, (float)(y + hh));
    const double sadxx = S((float)(x + 2 * hh), y);
    const double sadyy = S(x, (float)(y + 2 * hh));
    const double sadxy = S((float)(x + hh), (float)(y + hh));
    const float mdx = (float)((sadx - sad0) / hh), mdy = (float)((sady - sad0) / hh);
    const float mdxx = (float)(((sadxx - sadx) / hh - (sadx - sad0) / hh) / hh);
    const float mdyy = (float)(((sadyy - sady) / hh - (sady - sad0) / hh) / hh);
    const float mdxy = (float)(((sadxy - sady) / hh - (sadx - sad0) / hh) / hh);
    const float mdyx = (float)(((sadxy - sadx) / hh - (sady - sad0) / hh) / hh);
    const double H00 = mdxx, H01 = mdxy, H10 = mdyx, H11 = mdyy;
    const double det = H00 * H11 - H10 * H01;
    const double invdet = 1.0 / det;
    const double i00 = H11 * invdet, i10 = -H10 * invdet, i01 = -H01 * invdet, i11 = H00 * invdet;
    const double g0 = mdx, g1 = mdy;
    const double jj0 = i00 * g0 + i01 * g1, jj1 = i10 * g0 + i11 * g1;
    float dx = (float)-jj0, dy = (float)-jj1;
    if ((dx * dx + dy * dy) > 1) {
      dx /= std::sqrt(dx * dx + dy * dy);
      dy /= std::sqrt(dx * dx + dy * dy);
    }
    const float cx = (dx < 1.f) ? dx : 1.f, cy = (dy < 1.f) ? dy : 1.f;
    x += (-1.f < cx) ? cx : -1.f;
    y += (-1.f < cy) ? cy : -1.f;
    if (std::fabs(dx) < threshold / 10. && std::fabs(dy) < threshold / 10.) {
      ++it;
      break;
    }
  }
  if (iters) *iters += it;
  *px = x;
  *py = y;
  return 0;
}

// klt.h:403-424 TrackFeature: every pyramid level, threshold x 50 on the coarse levels.
int KltTrackFeature(const Tracker& T, const std::vector<Level>& src, const std::vector<Level>& dst, float sx, float sy,
                    float threshold, int max_iterations, float* px, float* py, int* iters) {
  const int lvls = (int)dst.size();
  std::vector<Patch> patches(lvls);
  float tx = sx, ty = sy;
  for (int i = 0; i < lvls; ++i) {
    patches[i] = PlainPatch(T, src[i].img, src[i].w, src[i].h, tx, ty, true);
    tx = (float)(tx * 0.5);
    ty = (float)(ty * 0.5);
  }
  const double s = 1. / (1 << (lvls - 1));
  float x = (float)(*px * s), y = (float)(*py * s);
  for (int i = lvls - 1; i > 0; --i) {
    const int st = KltTrack(T, dst[i], patches[i], threshold * 50, max_iterations, &x, &y, iters);
    if (st) return st;
    x = (float)(x * 2.);
    y = (float)(y * 2.);
  }
  const int st = KltTrack(T, dst[0], patches[0], threshold, max_iterations, &x, &y, iters);
  if (st) return st;
  *px = x;
  *py = y;
  return 0;
}

// brute.h:82-94 SADPatches(template, candidate): lighting-normalised, unmasked, sequential sum.
float BruteScore(const Tracker& T, const Patch& p1, const Patch& p2) {
  const float alpha = std::sqrt(p1.sumsq / p2.sumsq);
  const float beta = p1.mean - alpha * p2.mean;
  float sum = 0.f;
  for (int i = 0; i < T.len; ++i) {
    if (p1.data[i] == 0 || p2.data[i] == 0) continue;
    const float diff = p1.data[i] - p2.data[i] * alpha - beta;
    sum += std::fabs(diff * diff);
  }
  return sum;
}

// The float-stepped offsets of `for (float x = -window; x <= window; x += res)` (brute.h:104-105).
std::vector<float> BruteSteps(float window, float res) {
  std::vector<float> v;
  for (float x = -window; x <= window; x += res) v.push_back(x);
  return v;
}

// brute.h:96-117 SearchBest: exhaustive grid, x outer, y inner; a candidate replaces the best unless its
// score is larger (ties go to the later candidate).
float BruteSearchBest(const Tracker& T, const Level& L, const Patch& patch, float window, float res, float* ptx,
                      float* pty) {
  const std::vector<float> st = BruteSteps(window, res);
  const float p0x = *ptx, p0y = *pty;
  float best = 1e6f;
  for (float ox : st)
    for (float oy : st) {
      const float sad = BruteScore(T, patch, PlainPatch(T, L.img, L.w, L.h, p0x + ox, p0y + oy, false));
      if (sad > best) continue;
      *ptx = p0x + ox;
      *pty = p0y + oy;
      best = sad;
    }
  return best;
}

// brute.h:129-164 TrackFeature (threshold and max_iterations unused by the reference).
int BruteTrackFeature(const Tracker& T, const std::vector<Level>& src, const std::vector<Level>& dst, float sx,
                      float sy, float* px, float* py) {
  const int lvls = (int)dst.size();
  const float margin = 13;
  if (*px < margin || *py < margin || (*px + margin) > dst[0].w || (*py + margin) > dst[0].h) return 2;
  std::vector<Patch> patches(lvls);
  float tx = sx, ty = sy;
  for (int i = 0; i < lvls; ++i) {
    patches[i] = PlainPatch(T, src[i].img, src[i].w, src[i].h, tx, ty, false);
    tx = (float)(tx * 0.5);
    ty = (float)(ty * 0.5);
  }
  const double s = 1. / (1 << (lvls - 1));
  float x = (float)(*px * s), y = (float)(*py * s);
  for (int i = lvls - 1; i > 0; --i) {
    BruteSearchBest(T, dst[i], patches[i], 3, 1, &x, &y);
    const float sad = BruteSearchBest(T, dst[i], patches[i], 1, 0.33333f, &x, &y);
    if (sad > 100) return 2;
    x = (float)(x * 2.);
    y = (float)(y * 2.);
  }
  BruteSearchBest(T, dst[0], patches[0], 3, 1, &x, &y);
  BruteSearchBest(T, dst[0], patches[0], 1, 0.3333f, &x, &y);
  BruteSearchBest(T, dst[0], patches[0], 0.4f, 0.1f, &x, &y);
  BruteSearchBest(T, dst[0], patches[0], 0.2f, 0.025f, &x, &y);
  const float sad = BruteSearchBest(T, dst[0], patches[0], 8, 0.01f, &x, &y);
  if (sad > 100) return 2;
  *px = x;
  *py = y;
  return 0;
}

}  // namespace oracle_trk

extern "C" {

// MakePyramid of mode 0 (hessian.h), 1 (klt.h) or 2 (brute.h).
int ort_make_pyramid_mode(int mode, const uint8_t* bgr, int w, int h, int stride, int depth, float* out,
                          int32_t* dims) {
  if (mode == 0) return ort_make_pyramid(bgr, w, h, stride, depth, out, dims);
  oracle_trk::MakePyramidMode(mode, bgr, w, h, stride, depth, out, dims);
  return 0;
}

// One-directional TrackFeature of the mode for n features: templates GetPatches(from, from_xy), tracking on
// `to` from the initial guess in to_xy (updated only on success).  status: 0 OK, 2 OUT_OF_BOUNDS.  levels
// (mode 0 only; NULL = all levels): HessianTracker::GetPatches' level count.
int ort_track_feature_mode(int mode, const float* pyr_from, const float* pyr_to, const int32_t* dims, int depth, int win,
                           int n, const float* from_xy, float* to_xy, const int32_t* levels, float threshold,
                           int max_iterations, int32_t* status, int32_t* iters, int nthreads) {
  using namespace oracle_trk;
  std::vector<Level> from(depth), to(depth);
  size_t off = 0;
  for (int l = 0; l < depth; ++l) {
    from[l] = Level{pyr_from + off, dims[2 * l], dims[2 * l + 1]};
    to[l] = Level{pyr_to + off, dims[2 * l], dims[2 * l + 1]};
    off += (size_t)dims[2 * l] * dims[2 * l + 1];
  }
  Tracker T(win);
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int i = 0; i < n; ++i) {
    int it = 0;
    float x = to_xy[2 * i], y = to_xy[2 * i + 1];
    int st;
    if (mode == 0)
      st = TrackFeature(T, from, to, from_xy[2 * i], from_xy[2 * i + 1], levels ? levels[i] : depth, threshold,
                        max_iterations, &x, &y, &it);
    else if (mode == 1)
      st = KltTrackFeature(T, from, to, from_xy[2 * i], from_xy[2 * i + 1], threshold, max_iterations, &x, &y, &it);
    else
      st = BruteTrackFeature(T, from, to, from_xy[2 * i], from_xy[2 * i + 1], &x, &y);
    status[i] = st;
    if (iters) iters[i] = it;
    if (st == 0) {
      to_xy[2 * i] = x;
      to_xy[2 * i + 1] = y;
    }
  }
  return 0;
}

// brute.h SearchBest offsets of one (window, res) pass (checker of the device step tables).
int ort_brute_steps(float window, float res, float* out, int cap) {
  const std::vector<float> v = oracle_trk::BruteSteps(window, res);
  for (int i = 0; i < (int)v.size() && i < cap; ++i) out[i] = v[i];
  return (int)v.size();
}

}  // extern "C"
