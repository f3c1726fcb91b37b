// tracker.h — host driver of the device HessianTracker (one per sg_tracker handle).
#ifndef SG_TRACKER_H_
#define SG_TRACKER_H_

#include <hip/hip_runtime.h>

#include <vector>

#include "common.h"
#include "dbuf.h"

namespace sg {

constexpr int kTrkMaxDepth = 8;

// BGR u8 -> grey u8 with CV_RGB2GRAY's fixed-point weights on BGR memory (corners.hip).
__global__ void k_grey_u8(const uint8_t* bgr, int w, int h, int stride, uint8_t* grey);

struct TrackParams {
  int window, max_iterations;
  float threshold, fb_max;
  int retry_levels;
  const float* mask;
  unsigned long long* stamps = nullptr;   // diagnostics (SG_TRK_STAMP=1): per-phase cycles of the Newton loop
};
constexpr int kTrkStamps = 10;   // stage, probes, sums 1, score, sums 2 + differences, step, template, other, iters, waves

class Tracker {
 public:
  Tracker(const sg_tracker_options& o, const sg_device_options& d);
  ~Tracker();

  void SetImage(int slot, const uint8_t* bgr, int w, int h, int stride);
  void GetLevel(int slot, int level, float* out, int* w, int* h);
  void GetPatches(int slot, int level, int n, const float* xy, float* out, float* mean, float* sumsq);
  void LoadFeatures(int n, const float* from_xy, const float* to_xy, const int32_t* levels);
  void Run(int from, int to, int repeats);
  void Results(float* to_xy, int32_t* accepted, int32_t* iterations);
  // FindMatches (matcher.cpp:210-271) of n features into slot `to` in one launch: feature f's attempts are
  // aoff[f] .. aoff[f+1]-1, attempt a from slot aslot[a], match point axy[4a..4a+1], start axy[4a+2..4a+3];
  // which[f] = the accepted attempt's index in the feature's list or -1, to_xy its track.
  void FindMatches(int to, int n, const int32_t* aoff, const int32_t* aslot, const float* axy, const int32_t* levels,
                   float* to_xy, int32_t* which, int32_t* iterations);
  // One-directional TrackFeature of the configured FeatureTracker (hessian.h / klt.h / brute.h).
  void TrackFeature(int from, int to, int n, const float* from_xy, float* to_xy, const int32_t* levels,
                    int32_t* status, int32_t* iterations);
  // Matcher::Track's new-keyframe seeding (goodFeaturesToTrack + AddNewFeatures, corners.hip).
  void SeedFeatures(int slot, const float* match_xy, int nmatch, int max_corners, double quality, double min_distance,
                    float* corners_xy, int* ncorners, float* added_xy, int* nadded);
  double track_ms() const { return track_ms_; }
  // diagnostics: accumulated per-phase cycles of k_track_fb since the last call (SG_TRK_STAMP=1), kTrkStamps
  std::vector<unsigned long long> Stamps();
  double pyramid_ms() const { return pyr_ms_; }

 private:
  struct Slot {
    DBuf<float> pyr;
    DBuf<uint8_t> table;   // per-level {image, width, height} for the tracking kernel
    DBuf<uint8_t> grey;    // level-0 grey u8 (cvtColor RGB2GRAY) for corner seeding
    std::vector<int> w, h;
    std::vector<size_t> off;
    bool valid = false;
  };
  sg_tracker_options opt_;
  sg_device_options dev_;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_[4] = {nullptr, nullptr, nullptr, nullptr};
  std::vector<Slot> slots_;
  DBuf<float> mask_, tmp_, tmp2_;
  DBuf<uint8_t> img_;
  DBuf<float> from_, init_, out_;
  DBuf<int32_t> levels_, acc_, its_;
  std::vector<uint8_t> tabs_h_;   // every slot's level table [max_images][kTrkMaxDepth] (k_find_matches)
  DBuf<uint8_t> tabs_;
  DBuf<int32_t> aoff_, aslot_;
  DBuf<float> axy_;
  DBuf<float> seed_dx_, seed_dy_, seed_eig_, seed_val_, seed_val2_;
  DBuf<uint8_t> seed_flag_, seed_tmp_;
  DBuf<int> seed_idx_, seed_idx2_, seed_misc_;
  DBuf<float> brute_steps_, brute_tmpl_, brute_sad_;
  DBuf<int> brute_idx_;
  DBuf<uint8_t> brute_state_;
  int n_ = 0;
  bool ran_ = false;
  bool stamp_on_ = false;
  DBuf<unsigned long long> stamps_;
  double track_ms_ = 0.0, pyr_ms_ = 0.0;
};

}  // namespace sg

#endif  // SG_TRACKER_H_
