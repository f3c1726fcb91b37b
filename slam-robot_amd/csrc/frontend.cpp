// frontend.cpp — Matcher::Track (matcher.cpp:301-405) over the device tracker: the per-frame front end's
// bookkeeping in host C++, every image operation (pyramid, forward/backward tracking with the 3 -> 6 level
// retry, corner seeding) on the device through sg::Tracker.
//
// The reference walks its live features one at a time (FindMatches, matcher.cpp:210-271): for each
// feature not yet matched, try its stored views in order and keep the first forward/backward-consistent
// track.  Features are independent, so here FindMatches is one device launch: a wave per feature walks that
// feature's attempts (its views, in order) and stops at the first accepted track.  The observations are
// then appended in feature order, which is the order the reference's loop adds them.
//
// Defined orders where the reference's are implementation details:
//   * Feature::matches is a map<View*, Point2f> (matcher.cpp:43): ordered by pointer value.  Here views are
//     tried in creation order (what ascending addresses of successive `new View` give in practice).
//   * The "Remove bad matches" loop (matcher.cpp:325-328) erases from the set it iterates (undefined
//     behaviour); here every feature whose point is no longer feature_usable() is removed.
//   * Frame::Unproject's quaternion inverse (Eigen conjugate / squaredNorm) sums x² + y² + z² + w² in
//     that order.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <vector>

#include "tracker.h"   // hip_runtime.h first: project_math.h uses __forceinline__
#include "common.h"
#include "project_math.h"

namespace sg {
namespace {

constexpr int kMinMatches = 40;       // matcher.cpp:336, 350
constexpr int kMaxViews = 4;          // matcher.cpp:398
constexpr double kInitialDepth = 2000;  // matcher.cpp:376
constexpr int kMaxCorners = 120;      // matcher.cpp:127
constexpr double kQuality = 0.01;     // matcher.cpp:128
constexpr double kMinDistance = 20;   // matcher.cpp:129

struct Pose {
  double q[4], t[3], k[7];
};

// Camera::PixelToPlane (localmap.h:55-78).
void PixelToPlane(const double* k, double px, double py, double* out) {
  double xp = px, yp = py;
  xp -= k[5];
  yp -= k[6];
  xp /= k[3];
  yp /= k[4];
  const double x0 = xp, y0 = yp;
  for (int i = 0; i < 3; ++i) {
    const double r2 = xp * xp + yp * yp;
    const double distort = 1. / (1.0 + r2 * (k[0] + r2 * (k[1] + r2 * k[2])));
    xp = x0 * distort;
    yp = y0 * distort;
  }
  out[0] = xp;
  out[1] = yp;
}

// Frame::Unproject (localmap.cpp:29-37): homogeneous (plane * d, d, 1), rotated by the inverse quaternion
// (Eigen: conjugate / squaredNorm, then _transformVector), translated, normalised as a 4-vector.
void Unproject(const Pose& f, const double* plane, double distance, double* X) {
  const double v[3] = {plane[0] * distance, plane[1] * distance, distance};
  const double n2 = f.q[0] * f.q[0] + f.q[1] * f.q[1] + f.q[2] * f.q[2] + f.q[3] * f.q[3];
  double qi[4] = {0, 0, 0, 0};
  if (n2 > 0) {
    qi[0] = -f.q[0] / n2;
    qi[1] = -f.q[1] / n2;
    qi[2] = -f.q[2] / n2;
    qi[3] = f.q[3] / n2;
  }
  double c0 = qi[1] * v[2] - qi[2] * v[1];
  double c1 = qi[2] * v[0] - qi[0] * v[2];
  double c2 = qi[0] * v[1] - qi[1] * v[0];
  c0 += c0;
  c1 += c1;
  c2 += c2;
  const double p[3] = {(v[0] + qi[3] * c0) + (qi[1] * c2 - qi[2] * c1) + f.t[0],
                       (v[1] + qi[3] * c1) + (qi[2] * c0 - qi[0] * c2) + f.t[1],
                       (v[2] + qi[3] * c2) + (qi[0] * c1 - qi[1] * c0) + f.t[2]};
  const double nrm = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2] + 1.0 * 1.0);
  X[0] = p[0] / nrm;
  X[1] = p[1] / nrm;
  X[2] = p[2] / nrm;
  X[3] = 1.0 / nrm;
}

}  // namespace

class Frontend {
 public:
  Frontend(const sg_tracker_options& o, const sg_device_options& d) {
    SG_REQUIRE(o.max_images >= kMaxViews + 1, SG_EINVAL, "the matcher needs max_images >= 5 pyramid slots");
    trk_.reset(new Tracker(o, d));
    for (int s = o.max_images - 1; s >= 0; --s) free_slots_.push_back(s);
  }

  int Track(const uint8_t* bgr, int w, int h, int stride, int frame, const sg_map_callbacks& cb,
            sg_frontend_stats* st) {
    SG_REQUIRE(w > 0 && h > 0 && bgr, SG_EINVAL, "empty image");   // CHECK_NE(img.size().width, 0)
    cb_ = &cb;
    *st = sg_frontend_stats{};
    batches_ = 0;

    // The new view's pyramid (matcher.cpp:319-322).  The slot goes back to the free list on every exit
    // unless the view is kept (a callback failing or an expired view must not leak it).
    SG_REQUIRE(!free_slots_.empty(), SG_EINVAL, "no free pyramid slot");
    View view{frame, free_slots_.back(), next_view_seq_++, w, h};
    free_slots_.pop_back();
    struct SlotGuard {
      std::vector<int>& free;
      int slot;
      bool kept = false;
      ~SlotGuard() {
        if (!kept) free.push_back(slot);
      }
    } guard{free_slots_, view.slot};
    trk_->SetImage(view.slot, bgr, w, h, stride);

    // Remove bad matches (matcher.cpp:325-328).
    for (auto it = features_.begin(); it != features_.end();) {
      double X[4], unc;
      int32_t usable = 0;
      Call(cb.point_state(cb.user, it->second.point, X, &unc, &usable), "point_state");
      it = usable ? std::next(it) : features_.erase(it);
    }

    std::map<int, std::pair<float, float>> matches;   // feature id -> to_pt
    FindMatches(view, &matches);
    st->matches_first = (int)matches.size();
    if ((int)matches.size() < kMinMatches && cb.update_frames) {
      int32_t updated = 0;
      Call(cb.update_frames(cb.user, &updated), "update_frames");
      if (updated) FindMatches(view, &matches);
    }
    st->matches = (int)matches.size();
    st->track_batches = batches_;

    if ((int)matches.size() >= kMinMatches) {
      Finish(st);                          // the view is not kept (matcher.cpp:350-351): the guard frees its slot
      return 1;
    }

    // New keyframe: keep the matches and the view (matcher.cpp:354-362).
    st->keyframe = 1;
    Call(cb.set_keyframe(cb.user, frame), "set_keyframe");
    std::vector<float> mxy;
    mxy.reserve(2 * matches.size());
    for (auto& m : matches) {
      features_[m.first].matches.push_back({view.seq, m.second.first, m.second.second});
      mxy.push_back(m.second.first);
      mxy.push_back(m.second.second);
    }
    views_.push_back(view);
    guard.kept = true;   // the slot now belongs to the kept view

    // AddNewFeatures (matcher.cpp:123-169) and the new points (matcher.cpp:368-392).
    std::vector<float> corners(2 * kMaxCorners), added(2 * kMaxCorners);
    int nc = 0, na = 0;
    trk_->SeedFeatures(view.slot, mxy.empty() ? nullptr : mxy.data(), (int)matches.size(), kMaxCorners, kQuality,
                       kMinDistance, corners.data(), &nc, added.data(), &na);
    st->corners = nc;
    st->added = na;
    Pose pose;
    Call(cb.frame_pose(cb.user, frame, pose.q, pose.t, pose.k), "frame_pose");
    for (int i = 0; i < na; ++i) {
      const float px = added[2 * i], py = added[2 * i + 1];
      double plane[2], X[4];
      PixelToPlane(pose.k, (double)px, (double)py, plane);
      Unproject(pose, plane, kInitialDepth, X);
      const int id = next_fid_++;
      int32_t point = -1;
      Call(cb.add_point(cb.user, id, X, &point), "add_point");
      Call(cb.add_observation(cb.user, frame, (double)px, (double)py, point), "add_observation");
      Feature f;
      f.point = point;
      f.matches.push_back({view.seq, px, py});
      features_[id] = std::move(f);
    }

    // Potentially remove an old view (matcher.cpp:397-403).
    if ((int)views_.size() > kMaxViews) {
      const View old = views_.front();
      views_.erase(views_.begin());
      for (auto& f : features_) {
        auto& v = f.second.matches;
        for (size_t j = 0; j < v.size(); ++j)
          if (v[j].view_seq == old.seq) {
            v.erase(v.begin() + j);
            break;
          }
      }
      free_slots_.push_back(old.slot);
    }
    Finish(st);
    return 1;
  }

  int Features(int32_t* points, int32_t* ids, int cap) const {
    int i = 0;
    for (auto& f : features_) {
      if (i < cap) {
        if (points) points[i] = f.second.point;
        if (ids) ids[i] = f.first;
      }
      ++i;
    }
    return i;
  }

 private:
  struct View {
    int frame, slot;
    long long seq;
    int w, h;
  };
  struct Match {
    long long view_seq;
    float x, y;
  };
  struct Feature {
    int point = -1;
    std::vector<Match> matches;   // view creation order
  };

  static void Call(int32_t rc, const char* what) {
    SG_REQUIRE(rc == 0, SG_EINVAL, std::string("map callback ") + what + " failed");
  }

  const View* FindView(long long seq) const {
    for (auto& v : views_)
      if (v.seq == seq) return &v;
    return nullptr;
  }

  void Finish(sg_frontend_stats* st) {
    st->features = (int)features_.size();
    st->views = (int)views_.size();
  }

  // FindMatches (matcher.cpp:210-271) for every feature not yet in `matches`, batched in rounds.
  void FindMatches(const View& to, std::map<int, std::pair<float, float>>* matches) {
    Pose pose;
    Call(cb_->frame_pose(cb_->user, to.frame, pose.q, pose.t, pose.k), "frame_pose");
    struct Cand {
      int id;
      int levels;
      bool projected;
      float px, py;       // projected starting point
    };
    std::vector<Cand> active;
    for (auto& f : features_) {
      if (matches->count(f.first)) continue;
      double X[4], unc;
      int32_t usable;
      Call(cb_->point_state(cb_->user, f.second.point, X, &unc, &usable), "point_state");
      Cand c{f.first, unc > 100 ? 6 : 3, false, 0.f, 0.f};
      if (unc < 100) {
        double uv[2];
        if (Project(pose.q, pose.t, pose.k, X, uv)) {
          c.projected = true;
          c.px = (float)uv[0];
          c.py = (float)uv[1];
        }
      }
      active.push_back(c);
    }

    // Every feature's attempts in its view order (the out-of-bounds test of matcher.cpp:245-247 — note '>' for y
    // — drops a start before the device sees it), all features in one device launch (Tracker::FindMatches: a
    // wave per feature stops at its first forward/backward-consistent track).
    std::vector<int32_t> aoff(1, 0), aslot, lv;
    std::vector<float> axy;
    for (auto& c : active) {
      for (const Match& m : features_[c.id].matches) {
        const View* from = FindView(m.view_seq);
        SG_REQUIRE(from, SG_EINVAL, "feature refers to an expired view");
        const float tx = c.projected ? c.px : m.x, ty = c.projected ? c.py : m.y;
        if (tx < 0 || ty < 0 || tx >= (float)to.w || ty > (float)to.h) continue;
        aslot.push_back(from->slot);
        axy.insert(axy.end(), {m.x, m.y, tx, ty});
      }
      aoff.push_back((int32_t)aslot.size());
      lv.push_back(c.levels);
    }
    std::map<int, std::pair<float, float>> found;
    const int n = (int)active.size();
    if (n > 0 && aoff.back() > 0) {
      std::vector<float> to_xy(2 * (size_t)n);
      std::vector<int32_t> which(n, -1);
      trk_->FindMatches(to.slot, n, aoff.data(), aslot.data(), axy.data(), lv.data(), to_xy.data(), which.data(),
                        nullptr);
      ++batches_;
      for (int i = 0; i < n; ++i)
        if (which[i] >= 0) found[active[i].id] = {to_xy[2 * i], to_xy[2 * i + 1]};
    }
    // Add the new observations in the reference's loop order (features by id).
    for (auto& m : found) {
      (*matches)[m.first] = m.second;
      Call(cb_->add_observation(cb_->user, to.frame, (double)m.second.first, (double)m.second.second,
                                features_[m.first].point),
           "add_observation");
    }
  }

  std::unique_ptr<Tracker> trk_;
  std::vector<int> free_slots_;
  std::vector<View> views_;                  // deque<unique_ptr<View>> views (matcher.cpp:55)
  std::map<int, Feature> features_;          // FeatureSet ordered by point id (matcher.cpp:46-52)
  int next_fid_ = 0;                         // matcher.cpp:57
  long long next_view_seq_ = 0;
  const sg_map_callbacks* cb_ = nullptr;
  int batches_ = 0;
};

}  // namespace sg

struct sg_frontend {
  std::unique_ptr<sg::Frontend> f;
};

extern "C" {

int sg_frontend_create(sg_frontend** out, const sg_tracker_options* o, const sg_device_options* dev) {
  SG_CAPI_BEGIN
  SG_REQUIRE(out, SG_EINVAL, "null output handle");
  sg_tracker_options opt;
  sg_tracker_options_default(&opt);
  if (o) opt = *o;
  sg_device_options d;
  sg_device_options_default(&d);
  if (dev) d = *dev;
  auto h = std::make_unique<sg_frontend>();
  h->f.reset(new sg::Frontend(opt, d));
  *out = h.release();
  SG_CAPI_END
}

void sg_frontend_destroy(sg_frontend* f) { delete f; }

int sg_frontend_track(sg_frontend* f, const uint8_t* bgr, int32_t width, int32_t height, int32_t stride,
                      int32_t frame, int32_t camera, const sg_map_callbacks* cb, int32_t* result,
                      sg_frontend_stats* stats) {
  SG_CAPI_BEGIN
  (void)camera;   // only printed by the reference (matcher.cpp:366)
  SG_REQUIRE(f && cb && cb->frame_pose && cb->point_state && cb->add_point && cb->add_observation &&
                 cb->set_keyframe,
             SG_EINVAL, "null handle or callback");
  sg_frontend_stats st;
  const int r = f->f->Track(bgr, width, height, stride, frame, *cb, &st);
  if (result) *result = r;
  if (stats) *stats = st;
  SG_CAPI_END
}

int sg_frontend_features(sg_frontend* f, int32_t* points, int32_t* ids, int32_t* n) {
  SG_CAPI_BEGIN
  SG_REQUIRE(f && n, SG_EINVAL, "null argument");
  *n = f->f->Features(points, ids, *n);
  SG_CAPI_END
}

}  // extern "C"
