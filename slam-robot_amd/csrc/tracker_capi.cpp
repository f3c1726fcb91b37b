// tracker_capi.cpp — extern "C" entry points of the device HessianTracker (include/slamgpu.h, sg_tracker_*).
#include <memory>

#include "common.h"
#include "tracker.h"

struct sg_tracker {
  std::unique_ptr<sg::Tracker> t;
};

extern "C" {

void sg_tracker_options_default(sg_tracker_options* o) {
  if (!o) return;
  *o = sg_tracker_options{};
  o->window = 13;          // kWindowSize, matcher.cpp:27
  o->depth = 6;            // MakePyramid(img, 6), matcher.cpp:221
  o->max_iterations = 10;  // matcher.cpp:176
  o->threshold = 0.001f;   // matcher.cpp:176
  o->fb_max = 0.3f;        // matcher.cpp:200
  o->retry_levels = 6;     // matcher.cpp:248
  o->max_images = 8;
}

int sg_tracker_create(sg_tracker** out, const sg_tracker_options* o, const sg_device_options* dev) {
  SG_CAPI_BEGIN
  SG_REQUIRE(out, SG_EINVAL, "null output handle");
  sg_tracker_options opt;
  sg_tracker_options_default(&opt);
  if (o) opt = *o;
  sg_device_options d;
  sg_device_options_default(&d);
  if (dev) d = *dev;
  auto h = std::make_unique<sg_tracker>();
  h->t.reset(new sg::Tracker(opt, d));
  *out = h.release();
  SG_CAPI_END
}

void sg_tracker_destroy(sg_tracker* t) { delete t; }

int sg_tracker_set_image(sg_tracker* t, int32_t slot, const uint8_t* bgr, int32_t width, int32_t height,
                         int32_t stride) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t, SG_EINVAL, "null handle");
  t->t->SetImage(slot, bgr, width, height, stride);
  SG_CAPI_END
}

int sg_tracker_get_level(sg_tracker* t, int32_t slot, int32_t level, float* out, int32_t* width, int32_t* height) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t && width && height, SG_EINVAL, "null argument");
  int w = 0, h = 0;
  t->t->GetLevel(slot, level, out, &w, &h);
  *width = w;
  *height = h;
  SG_CAPI_END
}

int sg_tracker_get_patches(sg_tracker* t, int32_t slot, int32_t level, int32_t n, const float* xy, float* out,
                           float* mean, float* sumsq) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t && (n == 0 || (xy && out && mean && sumsq)), SG_EINVAL, "null argument");
  t->t->GetPatches(slot, level, n, xy, out, mean, sumsq);
  SG_CAPI_END
}

int sg_tracker_track(sg_tracker* t, int32_t from, int32_t to, int32_t n, const float* from_xy, float* to_xy,
                     const int32_t* levels, int32_t* accepted, int32_t* iterations) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t && (n == 0 || (from_xy && to_xy && accepted)), SG_EINVAL, "null argument");
  t->t->LoadFeatures(n, from_xy, to_xy, levels);
  t->t->Run(from, to, 1);
  t->t->Results(to_xy, accepted, iterations);
  SG_CAPI_END
}

int sg_tracker_load_features(sg_tracker* t, int32_t n, const float* from_xy, const float* to_xy,
                             const int32_t* levels) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t, SG_EINVAL, "null handle");
  t->t->LoadFeatures(n, from_xy, to_xy, levels);
  SG_CAPI_END
}

int sg_tracker_run(sg_tracker* t, int32_t from, int32_t to, int32_t repeats) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t, SG_EINVAL, "null handle");
  t->t->Run(from, to, repeats);
  SG_CAPI_END
}

int sg_tracker_results(sg_tracker* t, float* to_xy, int32_t* accepted, int32_t* iterations) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t, SG_EINVAL, "null handle");
  t->t->Results(to_xy, accepted, iterations);
  SG_CAPI_END
}

// Diagnostic (not in the public header): per-phase Newton-loop cycles of k_track_fb (SG_TRK_STAMP=1), summed
// over the waves since the last call: stage, probes, sums 1, score, sums 2, step, template, other, iterations,
// waves.
int sg_tracker_debug_stamps(sg_tracker* t, unsigned long long* out, int32_t n) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t && out, SG_EINVAL, "null argument");
  auto v = t->t->Stamps();
  for (int32_t i = 0; i < n && i < (int32_t)v.size(); ++i) out[i] = v[i];
  SG_CAPI_END
}

int sg_tracker_kernel_ms(sg_tracker* t, double* track_ms, double* pyramid_ms) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t, SG_EINVAL, "null handle");
  if (track_ms) *track_ms = t->t->track_ms();
  if (pyramid_ms) *pyramid_ms = t->t->pyramid_ms();
  SG_CAPI_END
}

int sg_tracker_seed_features(sg_tracker* t, int32_t slot, const float* match_xy, int32_t num_matches,
                             int32_t max_corners, double quality, double min_distance, float* corners_xy,
                             int32_t* num_corners, float* added_xy, int32_t* num_added) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t && corners_xy && num_corners && added_xy && num_added, SG_EINVAL, "null argument");
  int nc = 0, na = 0;
  t->t->SeedFeatures(slot, match_xy, num_matches, max_corners, quality, min_distance, corners_xy, &nc, added_xy, &na);
  *num_corners = nc;
  *num_added = na;
  SG_CAPI_END
}

int sg_tracker_track_feature(sg_tracker* t, int32_t from, int32_t to, int32_t n, const float* from_xy, float* to_xy,
                             const int32_t* levels, int32_t* status, int32_t* iterations) {
  SG_CAPI_BEGIN
  SG_REQUIRE(t, SG_EINVAL, "null handle");
  t->t->TrackFeature(from, to, n, from_xy, to_xy, levels, status, iterations);
  SG_CAPI_END
}

}  // extern "C"
