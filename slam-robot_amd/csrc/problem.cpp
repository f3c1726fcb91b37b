// problem.cpp — host side of the drop-in boundary: LocalMap SoA -> compact BA problem.
//
// Implements the frame / point selection rules of Slam::SolveFrames (slam.cpp:417-443),
// Slam::SolveAllFrames (slam.cpp:447-480) and Slam::SetupProblem (slam.cpp:257-414) on the sg_map view of
// a LocalMap, producing the sg_problem the device solver consumes.  Ceres keeps pointers into the map;
// here the solved blocks are copied back by sg_problem_write_back (same observable effect).
#include <algorithm>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "common.h"

namespace sg {

static thread_local std::string g_last_error;
void SetError(const std::string& msg) { g_last_error = msg; }

namespace {

struct ProblemStorage {
  std::vector<double> k, q, t, X, obs_pt;
  std::vector<int32_t> frame_camera, frame_map_index, point_map_index, obs_frame, obs_point, dist_frame,
      dist_prev;
  std::vector<uint8_t> frame_rot_free, frame_trans_free, point_free;

  void Clear() {
    for (auto* v : {&k, &q, &t, &X, &obs_pt}) v->clear();
    for (auto* v : {&frame_camera, &frame_map_index, &point_map_index, &obs_frame, &obs_point, &dist_frame, &dist_prev})
      v->clear();
    for (auto* v : {&frame_rot_free, &frame_trans_free, &point_free}) v->clear();
  }

  void Bind(sg_problem* p) {
    p->k = k.data();
    p->q = q.data();
    p->t = t.data();
    p->frame_camera = frame_camera.data();
    p->frame_rot_free = frame_rot_free.data();
    p->frame_trans_free = frame_trans_free.data();
    p->frame_map_index = frame_map_index.data();
    p->X = X.data();
    p->point_free = point_free.data();
    p->point_map_index = point_map_index.data();
    p->obs_pt = obs_pt.data();
    p->obs_frame = obs_frame.data();
    p->obs_point = obs_point.data();
    p->dist_frame = dist_frame.data();
    p->dist_prev = dist_prev.data();
    p->num_frames = (int32_t)frame_camera.size();
    p->num_points = (int32_t)point_free.size();
    p->num_obs = (int32_t)obs_frame.size();
    p->num_dist = (int32_t)dist_frame.size();
    p->num_cameras = (int32_t)(k.size() / 7);
    p->owner_ = this;
  }
};

// A freed problem's storage is kept for the thread's next problem (main.cpp builds one per SolveFrames call,
// each about the size of the last): its vectors keep their capacity, so a build neither allocates nor
// page-faults.  Build's scratch arrays are kept the same way.
constexpr size_t kStoragePool = 2;
thread_local std::vector<std::unique_ptr<ProblemStorage>> t_pool;

ProblemStorage* TakeStorage() {
  if (t_pool.empty()) return new ProblemStorage;
  ProblemStorage* st = t_pool.back().release();
  t_pool.pop_back();
  st->Clear();
  return st;
}

void ReturnStorage(ProblemStorage* st) {
  if (t_pool.size() < kStoragePool)
    t_pool.emplace_back(st);
  else
    delete st;
}

struct BuildScratch {
  std::vector<uint8_t> frame_used, point_in, point_fluid;
  std::vector<int32_t> obs_in, point_index, pts, frame_index;
};
thread_local BuildScratch t_scratch;

constexpr int kUnusableMask = (1 << SG_BAD_LOCATION) | (1 << SG_NO_BASELINE) | (1 << SG_NO_OBSERVATIONS) |
                              (1 << SG_BAD_FEATURE);  // TrackedPoint::slam_usable, localmap.h:242-248

// Validates the map; returns whether its observations are ordered by frame (a LocalMap's are: each frame's
// observations are appended when the frame is tracked), which lets Build walk only the presented frames' range.
bool CheckMap(const sg_map* m) {
  SG_REQUIRE(m != nullptr, SG_EINVAL, "null map");
  SG_REQUIRE(m->num_frames >= 0 && m->num_points >= 0 && m->num_obs >= 0 && m->num_cameras >= 0, SG_EINVAL,
             "negative map sizes");
  for (int32_t f = 0; f < m->num_frames; ++f) {
    SG_REQUIRE(m->frame_camera[f] >= 0 && m->frame_camera[f] < m->num_cameras, SG_EINVAL,
               "frame_camera out of range");
    SG_REQUIRE(m->frame_prev[f] >= -1 && m->frame_prev[f] < m->num_frames, SG_EINVAL, "frame_prev out of range");
  }
  // one branch-free sweep (the range tests and the order test accumulate), then the failing index if any
  const uint32_t F = (uint32_t)m->num_frames, P = (uint32_t)m->num_points;
  bool bad = false, sorted = true;
  int32_t prev = 0;
  for (int32_t o = 0; o < m->num_obs; ++o) {
    const int32_t f = m->obs_frame[o];
    bad |= ((uint32_t)f >= F) | ((uint32_t)m->obs_point[o] >= P);
    sorted &= f >= prev;
    prev = f;
  }
  if (bad)
    for (int32_t o = 0; o < m->num_obs; ++o) {
      SG_REQUIRE(m->obs_frame[o] >= 0 && m->obs_frame[o] < m->num_frames, SG_EINVAL, "obs_frame out of range");
      SG_REQUIRE(m->obs_point[o] >= 0 && m->obs_point[o] < m->num_points, SG_EINVAL, "obs_point out of range");
    }
  return sorted;
}

// role[f]: 0 = not presented, 1 = presented & solved, 2 = presented & constant.
bool Build(const sg_map* m, const std::vector<uint8_t>& role, double range, bool cameras_free, bool obs_by_frame,
           sg_problem* out) {
  const int F = m->num_frames, P = m->num_points, M = m->num_obs;
  // Observations to visit: all of them, or (observations ordered by frame) the range of the presented frames.
  int o_lo = 0, o_hi = M;
  if (obs_by_frame) {
    int fmin = F, fmax = -1;
    for (int f = 0; f < F; ++f)
      if (role[f]) {
        fmin = std::min(fmin, f);
        fmax = std::max(fmax, f);
      }
    o_lo = (int)(std::lower_bound(m->obs_frame, m->obs_frame + M, fmin) - m->obs_frame);
    o_hi = (int)(std::upper_bound(m->obs_frame + o_lo, m->obs_frame + M, fmax) - m->obs_frame);
  }
  // Pass 1 (slam.cpp:274-303): usable observations of presented frames, in map order (branch-free: the
  // selection is data-dependent, so the marks are or-ed in and the list is compacted by its running count).
  BuildScratch& sc = t_scratch;
  std::vector<uint8_t>&frame_used = sc.frame_used, &point_in = sc.point_in, &point_fluid = sc.point_fluid;
  frame_used.assign(F, 0);
  point_in.assign(P, 0);
  point_fluid.assign(P, 0);
  std::vector<int32_t>& obs_in = sc.obs_in;
  obs_in.resize(std::max(o_hi - o_lo, 0));
  size_t nin = 0;
  for (int o = o_lo; o < o_hi; ++o) {
    const int f = m->obs_frame[o], pt = m->obs_point[o];
    const uint8_t use = (role[f] != 0) & (m->obs_disabled[o] == 0) & ((m->point_flags[pt] & kUnusableMask) == 0);
    obs_in[nin] = o;
    nin += use;
    frame_used[f] |= use;
    point_in[pt] |= use;
    point_fluid[pt] |= use & (role[f] == 1);
  }
  int used = 0;
  for (int f = 0; f < F; ++f) {
    used += role[f] != 0 && frame_used[f];
  }
  if (used < 2) return false;  // "Slam aborted due to frame set too small" (slam.cpp:305-308)

  auto* st = TakeStorage();
  std::vector<int32_t>& frame_index = sc.frame_index;
  frame_index.assign(F, -1);
  auto add_frame = [&](int f, bool rot_free, bool trans_free) {
    frame_index[f] = (int32_t)st->frame_camera.size();
    st->frame_camera.push_back(m->frame_camera[f]);
    st->frame_map_index.push_back(f);
    st->frame_rot_free.push_back(rot_free);
    st->frame_trans_free.push_back(trans_free);
    st->q.insert(st->q.end(), m->q + 4 * f, m->q + 4 * f + 4);
    st->t.insert(st->t.end(), m->t + 3 * f, m->t + 3 * f + 3);
  };
  // Used frames become quaternion + translation blocks, constant when not solved (slam.cpp:314-333).
  for (int f = 0; f < F; ++f)
    if (role[f] && frame_used[f]) add_frame(f, role[f] == 1, role[f] == 1);
  // FrameDistance between every solved, used frame and its presented previous frame (slam.cpp:383-411).
  // A presented but unused previous frame contributes a fresh (free) translation block.
  for (int f = 0; f < F; ++f) {
    if (role[f] != 1 || !frame_used[f]) continue;
    const int prev = m->frame_prev[f];
    if (prev < 0 || !role[prev]) continue;
    if (frame_index[prev] < 0) add_frame(prev, false, true);
    st->dist_frame.push_back(frame_index[f]);
    st->dist_prev.push_back(frame_index[prev]);
  }
  // Points (slam.cpp:345-354).
  std::vector<int32_t>&point_index = sc.point_index, &pts = sc.pts;
  point_index.assign(P, -1);
  pts.resize(P);
  size_t npt = 0;
  for (int pt = 0; pt < P; ++pt) {   // compaction of the marked points, in map order
    pts[npt] = pt;
    npt += point_in[pt];
  }
  st->point_map_index.assign(pts.begin(), pts.begin() + npt);
  st->point_free.resize(npt);
  st->X.resize(4 * npt);
  for (size_t i = 0; i < npt; ++i) {
    const int pt = pts[i];
    point_index[pt] = (int32_t)i;
    const bool is_const = m->point_uncertainty[pt] <= 100.0 && !point_fluid[pt];
    st->point_free[i] = !is_const;
    std::memcpy(st->X.data() + 4 * i, m->X + 4 * (size_t)pt, 4 * sizeof(double));
  }
  st->obs_pt.resize(2 * nin);
  st->obs_frame.resize(nin);
  st->obs_point.resize(nin);
  for (size_t i = 0; i < nin; ++i) {
    const int o = obs_in[i];
    st->obs_pt[2 * i] = m->obs_pt[2 * o];
    st->obs_pt[2 * i + 1] = m->obs_pt[2 * o + 1];
    st->obs_frame[i] = frame_index[m->obs_frame[o]];
    st->obs_point[i] = point_index[m->obs_point[o]];
  }
  st->k.assign(m->k, m->k + 7 * m->num_cameras);
  std::memset(out, 0, sizeof(*out));
  st->Bind(out);
  out->cameras_free = cameras_free ? 1 : 0;
  out->range = range;
  out->dist_target = 150.0;  // slam.cpp:403
  out->dist_range = 15.0;    // slam.cpp:404
  out->stab_range = 5.0;     // slam.cpp:463
  return true;
}

void CheckProblem(const sg_problem* p) {
  SG_REQUIRE(p != nullptr, SG_EINVAL, "null problem");
  for (int32_t o = 0; o < p->num_obs; ++o) {
    SG_REQUIRE(p->obs_frame[o] >= 0 && p->obs_frame[o] < p->num_frames, SG_EINVAL, "obs_frame out of range");
    SG_REQUIRE(p->obs_point[o] >= 0 && p->obs_point[o] < p->num_points, SG_EINVAL, "obs_point out of range");
  }
  for (int32_t d = 0; d < p->num_dist; ++d)
    SG_REQUIRE(p->dist_frame[d] >= 0 && p->dist_frame[d] < p->num_frames && p->dist_prev[d] >= 0 &&
                   p->dist_prev[d] < p->num_frames,
               SG_EINVAL, "FrameDistance frame out of range");
  for (int32_t f = 0; f < p->num_frames; ++f)
    SG_REQUIRE(p->frame_camera[f] >= 0 && p->frame_camera[f] < p->num_cameras, SG_EINVAL,
               "frame_camera out of range");
}

}  // namespace

void ValidateProblem(const sg_problem* p) { CheckProblem(p); }

}  // namespace sg

extern "C" {

const char* sg_version(void) { return "slamgpu 0.1 (gfx950)"; }
const char* sg_last_error(void) { return sg::g_last_error.c_str(); }

void sg_solver_options_default(sg_solver_options* o) {
  o->max_num_iterations = 1000;     // slam.cpp:493
  o->function_tolerance = 1e-7;     // slam.cpp:494
  o->gradient_tolerance = 1e-10;    // Ceres 1.8 defaults below
  o->parameter_tolerance = 1e-8;
  o->min_relative_decrease = 1e-3;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
  o->disable_termination = 0;
  o->always_linearize = 0;
}

void sg_device_options_default(sg_device_options* o) {
  o->device = 0;
  o->precision = 0;
  o->rank = 0;
  o->nranks = 1;
}

int sg_problem_from_map_frames(const sg_map* map, int32_t num_to_solve, int32_t num_to_present, double range,
                               sg_problem* out, int32_t* built) {
  SG_CAPI_BEGIN
  const bool obs_by_frame = sg::CheckMap(map);
  SG_REQUIRE(out && built, SG_EINVAL, "null output");
  // slam.cpp:423-434: the newest num_to_solve frames are solved, the next ones up to num_to_present are
  // presented as constant.
  std::vector<uint8_t> role(map->num_frames, 0);
  for (int i = 0; i < map->num_frames; ++i) {
    const int f = map->num_frames - i - 1;
    if (i < num_to_solve) role[f] = 1;
    else if (i < num_to_present) role[f] = 2;
    else break;
  }
  *built = sg::Build(map, role, range, false, obs_by_frame, out) ? 1 : 0;
  SG_CAPI_END
}

int sg_problem_from_map_all(const sg_map* map, double range, int32_t solve_cameras, sg_problem* out,
                            int32_t* built) {
  SG_CAPI_BEGIN
  const bool obs_by_frame = sg::CheckMap(map);
  SG_REQUIRE(out && built, SG_EINVAL, "null output");
  std::vector<uint8_t> role(map->num_frames, 1);  // slam.cpp:449-452
  *built = sg::Build(map, role, range, solve_cameras != 0, obs_by_frame, out) ? 1 : 0;
  SG_CAPI_END
}

void sg_problem_free(sg_problem* p) {
  if (p && p->owner_) {
    sg::ReturnStorage(static_cast<sg::ProblemStorage*>(p->owner_));
    p->owner_ = nullptr;
  }
}

int sg_problem_write_back(const sg_problem* p, sg_map* map) {
  SG_CAPI_BEGIN
  SG_REQUIRE(p && map, SG_EINVAL, "null argument");
  for (int32_t f = 0; f < p->num_frames; ++f) {
    const int32_t mf = p->frame_map_index[f];
    SG_REQUIRE(mf >= 0 && mf < map->num_frames, SG_EINVAL, "frame_map_index out of range");
    std::memcpy(map->q + 4 * mf, p->q + 4 * f, 4 * sizeof(double));
    std::memcpy(map->t + 3 * mf, p->t + 3 * f, 3 * sizeof(double));
  }
  for (int32_t i = 0; i < p->num_points; ++i) {
    const int32_t mp = p->point_map_index[i];
    SG_REQUIRE(mp >= 0 && mp < map->num_points, SG_EINVAL, "point_map_index out of range");
    std::memcpy(map->X + 4 * mp, p->X + 4 * i, 4 * sizeof(double));
  }
  if (p->cameras_free) std::memcpy(map->k, p->k, 7 * sizeof(double) * map->num_cameras);
  SG_CAPI_END
}

// Landmark shard: points ordered by their first observing frame, split into nranks contiguous ranges of
// roughly equal observation count; each shard keeps every frame, camera and FrameDistance block.
int sg_problem_shard(const sg_problem* p, int32_t rank, int32_t nranks, sg_problem* out) {
  SG_CAPI_BEGIN
  sg::CheckProblem(p);
  SG_REQUIRE(out && nranks >= 1 && rank >= 0 && rank < nranks, SG_EINVAL, "bad shard arguments");
  const int P = p->num_points, M = p->num_obs;
  std::vector<int32_t> first(P, INT32_MAX), nobs(P, 0);
  for (int o = 0; o < M; ++o) {
    first[p->obs_point[o]] = std::min(first[p->obs_point[o]], p->obs_frame[o]);
    nobs[p->obs_point[o]]++;
  }
  std::vector<int32_t> order(P);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return first[a] < first[b]; });
  // Balanced split on observation counts.
  std::vector<int32_t> owner(P, 0);
  long long total = 0;
  for (int i = 0; i < P; ++i) total += nobs[i];
  long long acc = 0;
  for (int i = 0; i < P; ++i) {
    const int pt = order[i];
    int r = total > 0 ? (int)((acc * nranks) / total) : (int)((long long)i * nranks / std::max(P, 1));
    owner[pt] = std::min(r, nranks - 1);
    acc += nobs[pt];
  }
  auto* st = new sg::ProblemStorage;
  st->k.assign(p->k, p->k + 7 * p->num_cameras);
  st->q.assign(p->q, p->q + 4 * p->num_frames);
  st->t.assign(p->t, p->t + 3 * p->num_frames);
  st->frame_camera.assign(p->frame_camera, p->frame_camera + p->num_frames);
  st->frame_rot_free.assign(p->frame_rot_free, p->frame_rot_free + p->num_frames);
  st->frame_trans_free.assign(p->frame_trans_free, p->frame_trans_free + p->num_frames);
  st->frame_map_index.assign(p->frame_map_index, p->frame_map_index + p->num_frames);
  st->dist_frame.assign(p->dist_frame, p->dist_frame + p->num_dist);
  st->dist_prev.assign(p->dist_prev, p->dist_prev + p->num_dist);
  std::vector<int32_t> local(P, -1);
  for (int i = 0; i < P; ++i) {
    const int pt = order[i];
    if (owner[pt] != rank) continue;
    local[pt] = (int32_t)st->point_free.size();
    st->point_free.push_back(p->point_free[pt]);
    st->point_map_index.push_back(p->point_map_index[pt]);
    st->X.insert(st->X.end(), p->X + 4 * pt, p->X + 4 * pt + 4);
  }
  for (int o = 0; o < M; ++o) {
    const int pt = p->obs_point[o];
    if (owner[pt] != rank) continue;
    st->obs_pt.push_back(p->obs_pt[2 * o]);
    st->obs_pt.push_back(p->obs_pt[2 * o + 1]);
    st->obs_frame.push_back(p->obs_frame[o]);
    st->obs_point.push_back(local[pt]);
  }
  std::memset(out, 0, sizeof(*out));
  st->Bind(out);
  out->cameras_free = p->cameras_free;
  out->range = p->range;
  out->dist_target = p->dist_target;
  out->dist_range = p->dist_range;
  out->stab_range = p->stab_range;
  SG_CAPI_END
}

}  // extern "C"
