// oracle_ba.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement ("oracle") of the reference's local bundle-adjustment hot path.  It is linked only by
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker and the timed CPU
// baseline; the product library (libslamgpu.so) never links, loads or calls it.
//
// PARITY STATUS: "parity unpinned" by reference fixtures.  The reference (ywrt/slam-robot) cannot be
// compiled in this image (it needs Eigen, Ceres Solver 1.8.0, OpenCV 2.x, glog; none present or vendored)
// and its repository holds no golden vectors or tests for this path.  The Ceres 1.8.0
// algorithm (a third-party dependency pinned by Makefile:7-8, not vendored) is restated here from its
// published design.  The restatement is pinned instead by: known-answer projection tests, dual-number vs
// finite-difference Jacobian checks, and converged minima from an independent solver
// (scipy.optimize.least_squares, loss='cauchy'), all in tests/.
//
// What is restated (file:line into /root/reference):
//   ProjectPoint               project.h:11-54         (templated; evaluated on double and on Jet<18>)
//   ReprojectionError          slam.cpp:60-84
//   FrameDistance              slam.cpp:86-105, 383-411
//   CameraStabilization        slam.cpp:107-124, 459-471
//   Slam::SetupProblem         slam.cpp:257-414
//   Slam::SolveFrames          slam.cpp:417-443
//   Slam::SolveAllFrames       slam.cpp:447-480
//   Slam::Run                  slam.cpp:482-521  -> Ceres 1.8 TrustRegionMinimizer + LevenbergMarquardt
//                                                   strategy + SPARSE_SCHUR (Schur + dense Cholesky of S)
//   Slam::ReprojectMap         slam.cpp:523-548
// Ceres 1.8 pieces restated (not vendored): AutoDiffCostFunction (forward-mode dual numbers = Jet),
// CauchyLoss + Corrector (rho'' < 0 => scale by sqrt(rho')), QuaternionParameterization ([w,x,y,z]
// convention applied to Eigen [x,y,z,w] memory, slam.cpp:312-313), Jacobi column scaling (computed once
// from the initial Jacobian), LM diagonal clamp [1e-6,1e32], radius update, relative gradient tolerance,
// function/parameter tolerances, <=5 consecutive invalid steps, fixed-cost removal of all-constant
// residual blocks, summary.iterations bookkeeping (iteration 0 counted, terminating iteration not pushed).

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <limits>
#include <map>
#include <set>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "slamgpu.h"

namespace oracle {

// ------------------------------------------------------------------------------------------------
// Jet: forward-mode dual number, the stand-in for ceres::Jet used by AutoDiffCostFunction.
template <int N>
struct Jet {
  double a;
  double v[N];
  Jet() : a(0.0) { for (int i = 0; i < N; ++i) v[i] = 0.0; }
  explicit Jet(double x) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0.0; }
  Jet(double x, int k) : a(x) {
    for (int i = 0; i < N; ++i) v[i] = 0.0;
    v[k] = 1.0;
  }
};
template <int N> inline Jet<N> operator+(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> h; h.a = f.a + g.a; for (int i = 0; i < N; ++i) h.v[i] = f.v[i] + g.v[i]; return h; }
template <int N> inline Jet<N> operator-(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> h; h.a = f.a - g.a; for (int i = 0; i < N; ++i) h.v[i] = f.v[i] - g.v[i]; return h; }
template <int N> inline Jet<N> operator-(const Jet<N>& f) {
  Jet<N> h; h.a = -f.a; for (int i = 0; i < N; ++i) h.v[i] = -f.v[i]; return h; }
template <int N> inline Jet<N> operator*(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> h; h.a = f.a * g.a; for (int i = 0; i < N; ++i) h.v[i] = f.a * g.v[i] + f.v[i] * g.a; return h; }
template <int N> inline Jet<N> operator/(const Jet<N>& f, const Jet<N>& g) {
  // Ceres: g_inv = 1/g.a; f_over_g = f.a*g_inv; (f.v - f_over_g*g.v)*g_inv
  Jet<N> h; const double gi = 1.0 / g.a; h.a = f.a * gi;
  for (int i = 0; i < N; ++i) h.v[i] = (f.v[i] - h.a * g.v[i]) * gi; return h; }
template <int N> inline Jet<N> operator*(double s, const Jet<N>& f) {
  Jet<N> h; h.a = s * f.a; for (int i = 0; i < N; ++i) h.v[i] = s * f.v[i]; return h; }
template <int N> inline Jet<N> operator*(const Jet<N>& f, double s) { return s * f; }
template <int N> inline Jet<N> operator+(const Jet<N>& f, double s) { Jet<N> h = f; h.a += s; return h; }
template <int N> inline Jet<N> operator-(const Jet<N>& f, double s) { Jet<N> h = f; h.a -= s; return h; }
template <int N> inline Jet<N> sqrt(const Jet<N>& f) {
  Jet<N> h; h.a = std::sqrt(f.a); const double t = 1.0 / (2.0 * h.a);
  for (int i = 0; i < N; ++i) h.v[i] = f.v[i] * t; return h; }
template <int N> inline bool operator<(const Jet<N>& f, const Jet<N>& g) { return f.a < g.a; }
template <int N> inline double value(const Jet<N>& f) { return f.a; }
inline double value(double f) { return f; }
template <typename T> inline T mkconst(double x);
template <> inline double mkconst<double>(double x) { return x; }
template <> inline Jet<18> mkconst<Jet<18>>(double x) { return Jet<18>(x); }
template <> inline Jet<7> mkconst<Jet<7>>(double x) { return Jet<7>(x); }
template <> inline Jet<6> mkconst<Jet<6>>(double x) { return Jet<6>(x); }

// ------------------------------------------------------------------------------------------------
// project.h:11-54.  q is Eigen memory [x,y,z,w]; p = q * (X.xyz - t * X.w) uses Eigen's
// QuaternionBase::_transformVector: uv = 2 (q.vec x v);  p = v + w*uv + q.vec x uv.
template <typename T>
inline bool ProjectPoint(const T* q, const T* t, const T* k, const T* X, T* out) {
  const T v0 = X[0] - t[0] * X[3];
  const T v1 = X[1] - t[1] * X[3];
  const T v2 = X[2] - t[2] * X[3];
  T c0 = q[1] * v2 - q[2] * v1;
  T c1 = q[2] * v0 - q[0] * v2;
  T c2 = q[0] * v1 - q[1] * v0;
  c0 = c0 + c0; c1 = c1 + c1; c2 = c2 + c2;
  const T p0 = (v0 + q[3] * c0) + (q[1] * c2 - q[2] * c1);
  const T p1 = (v1 + q[3] * c1) + (q[2] * c0 - q[0] * c2);
  const T p2 = (v2 + q[3] * c2) + (q[0] * c1 - q[1] * c0);
  // project.h:27 — behind-camera rejection (the reference also printf()s here; we do not).
  if (value(p2) < 0.001 * value(X[3])) return false;
  T xp = p0 / p2;
  T yp = p1 / p2;
  const T r2 = xp * xp + yp * yp;
  const T distort = mkconst<T>(1.0) + r2 * (k[0] + r2 * (k[1] + r2 * k[2]));
  xp = xp * distort; yp = yp * distort;
  xp = xp * k[3]; yp = yp * k[4];
  xp = xp + k[5]; yp = yp + k[6];
  out[0] = xp; out[1] = yp;
  return true;
}

// ceres::CauchyLoss(a): b = a^2, c = 1/b; rho = [b log(1+s c), 1/(1+s c), -c/(1+s c)^2].
struct Cauchy {
  double b, c;
  explicit Cauchy(double a) : b(a * a), c(1.0 / (a * a)) {}
  void Evaluate(double s, double rho[3]) const {
    const double sum = 1.0 + s * c;
    const double inv = 1.0 / sum;
    rho[0] = b * std::log(sum);
    rho[1] = inv;
    rho[2] = -c * (inv * inv);
  }
};

// ceres::QuaternionParameterization (Ceres [w,x,y,z] convention, applied by the reference to Eigen
// [x,y,z,w] memory).  Plus and the 4x3 local Jacobian, row-major.
inline void QuatPlus(const double* x, const double* d, double* out) {
  const double nd = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd > 0.0) {
    const double s = std::sin(nd) / nd;
    const double z[4] = {std::cos(nd), s * d[0], s * d[1], s * d[2]};
    out[0] = z[0] * x[0] - z[1] * x[1] - z[2] * x[2] - z[3] * x[3];
    out[1] = z[0] * x[1] + z[1] * x[0] + z[2] * x[3] - z[3] * x[2];
    out[2] = z[0] * x[2] - z[1] * x[3] + z[2] * x[0] + z[3] * x[1];
    out[3] = z[0] * x[3] + z[1] * x[2] - z[2] * x[1] + z[3] * x[0];
  } else {
    for (int i = 0; i < 4; ++i) out[i] = x[i];
  }
}
inline void QuatLocalJacobian(const double* x, double* L) {
  L[0] = -x[1]; L[1] = -x[2]; L[2] = -x[3];
  L[3] = x[0];  L[4] = x[3];  L[5] = -x[2];
  L[6] = -x[3]; L[7] = x[0];  L[8] = x[1];
  L[9] = x[2];  L[10] = -x[1]; L[11] = x[0];
}

// ------------------------------------------------------------------------------------------------
// Problem assembly (slam.cpp:257-414) into an oracle-owned sg_problem.
struct OwnedProblem {
  std::vector<double> k, q, t, X, obs_pt;
  std::vector<int32_t> frame_camera, frame_map_index, point_map_index, obs_frame, obs_point, dist_frame,
      dist_prev;
  std::vector<uint8_t> frame_rot_free, frame_trans_free, point_free;
  sg_problem p;
  void Bind() {
    p.k = k.data(); p.q = q.data(); p.t = t.data(); p.frame_camera = frame_camera.data();
    p.frame_rot_free = frame_rot_free.data(); p.frame_trans_free = frame_trans_free.data();
    p.frame_map_index = frame_map_index.data(); p.X = X.data(); p.point_free = point_free.data();
    p.point_map_index = point_map_index.data(); p.obs_pt = obs_pt.data(); p.obs_frame = obs_frame.data();
    p.obs_point = obs_point.data(); p.dist_frame = dist_frame.data(); p.dist_prev = dist_prev.data();
    p.owner_ = nullptr;
  }
};

static bool SlamUsable(int flags) {  // localmap.h:242-248
  return !(flags & (1 << SG_BAD_LOCATION)) && !(flags & (1 << SG_NO_BASELINE)) &&
         !(flags & (1 << SG_NO_OBSERVATIONS)) && !(flags & (1 << SG_BAD_FEATURE));
}

// frames: map frame index -> is_const  (std::map<Frame*, bool> of slam.cpp:421/449)
static bool SetupProblem(const sg_map& m, double range, const std::map<int, bool>& frames, bool cameras_free,
                         OwnedProblem* out) {
  std::vector<std::vector<int>> frame_obs(m.num_frames);
  for (int o = 0; o < m.num_obs; ++o) frame_obs[m.obs_frame[o]].push_back(o);

  std::set<int> skip_frames, point_set, fluid_points;
  std::vector<int> used_obs;
  for (const auto& fr : frames) {
    const int f = fr.first;
    const bool is_const = fr.second;
    bool used = false;
    for (int o : frame_obs[f]) {
      if (m.obs_disabled[o]) continue;                                   // slam.cpp:280
      if (!SlamUsable(m.point_flags[m.obs_point[o]])) continue;          // slam.cpp:282
      used_obs.push_back(o);
      used = true;
      point_set.insert(m.obs_point[o]);
      if (!is_const) fluid_points.insert(m.obs_point[o]);
    }
    if (!used) skip_frames.insert(f);
  }
  if ((int)frames.size() - (int)skip_frames.size() < 2) return false;   // slam.cpp:305-308

  // Frames that become parameter blocks: used frames, plus skipped previous frames referenced by
  // FrameDistance (their translation becomes a free block, slam.cpp:383-411).
  std::map<int, int> fidx;
  auto add_frame = [&](int f, bool rot_free, bool trans_free) {
    auto it = fidx.find(f);
    if (it != fidx.end()) {
      out->frame_trans_free[it->second] |= trans_free;
      return it->second;
    }
    const int i = (int)out->frame_map_index.size();
    fidx[f] = i;
    out->frame_map_index.push_back(f);
    out->frame_camera.push_back(m.frame_camera[f]);
    out->frame_rot_free.push_back(rot_free);
    out->frame_trans_free.push_back(trans_free);
    for (int j = 0; j < 4; ++j) out->q.push_back(m.q[4 * f + j]);
    for (int j = 0; j < 3; ++j) out->t.push_back(m.t[3 * f + j]);
    return i;
  };
  for (const auto& fr : frames) {
    if (skip_frames.count(fr.first)) continue;
    add_frame(fr.first, !fr.second, !fr.second);                         // slam.cpp:323-333
  }
  // FrameDistance blocks.
  for (const auto& fr : frames) {
    if (fr.second) continue;
    if (skip_frames.count(fr.first)) continue;
    const int prev = m.frame_prev[fr.first];
    if (prev < 0 || !frames.count(prev)) continue;                       // slam.cpp:393-395
    const int a = fidx[fr.first];
    int b;
    if (skip_frames.count(prev)) b = add_frame(prev, false, true);       // new (free) translation block
    else b = fidx[prev];
    out->dist_frame.push_back(a);
    out->dist_prev.push_back(b);
  }
  // Points (slam.cpp:345-354): const iff uncertainty <= 100 and not referenced by a free frame.
  std::map<int, int> pidx;
  for (int pnt : point_set) {
    const int i = (int)out->point_map_index.size();
    pidx[pnt] = i;
    out->point_map_index.push_back(pnt);
    const bool is_const = (m.point_uncertainty[pnt] <= 100.0) && !fluid_points.count(pnt);
    out->point_free.push_back(!is_const);
    for (int j = 0; j < 4; ++j) out->X.push_back(m.X[4 * pnt + j]);
  }
  std::sort(used_obs.begin(), used_obs.end());
  for (int o : used_obs) {
    out->obs_pt.push_back(m.obs_pt[2 * o]);
    out->obs_pt.push_back(m.obs_pt[2 * o + 1]);
    out->obs_frame.push_back(fidx[m.obs_frame[o]]);
    out->obs_point.push_back(pidx[m.obs_point[o]]);
  }
  out->k.assign(m.k, m.k + 7 * m.num_cameras);
  out->Bind();
  sg_problem& p = out->p;
  p.num_cameras = m.num_cameras;
  p.cameras_free = cameras_free ? 1 : 0;
  p.num_frames = (int)out->frame_map_index.size();
  p.num_points = (int)out->point_map_index.size();
  p.num_obs = (int)out->obs_frame.size();
  p.num_dist = (int)out->dist_frame.size();
  p.range = range;
  p.dist_target = 150.0;
  p.dist_range = 15.0;
  p.stab_range = 5.0;
  return true;
}

// ------------------------------------------------------------------------------------------------
// The solver (Ceres 1.8 TrustRegionMinimizer + LevenbergMarquardtStrategy + SPARSE_SCHUR).
struct Options {
  sg_solver_options o;
  int nthreads;
};

struct ObsLin {
  double r[2];         // corrected residual  sqrt(rho') r
  double Jc[2][13];    // corrected camera-side local Jacobian: rot(3) trans(3) intrinsics(7)
  double Jp[2][4];     // corrected point Jacobian
  double cost;         // 0.5 rho
};

class Solver {
 public:
  Solver(sg_problem* p, const Options& opt) : p_(p), opt_(opt), cauchy_(p->range), dist_cauchy_(p->dist_range),
                                               stab_cauchy_(p->stab_range) {
    Layout();
  }

  // Returns summary (also writes solved blocks into p_).
  void Solve(sg_solver_summary* s);

  // Evaluate reprojection residuals at the current state (for parity tests): uncorrected r, cost.
  bool EvaluateResiduals(double* r_out, double* cost_out, int* nfail);

  // Unscaled reduced camera system at the current state, points damped by diag/radius, cameras
  // undamped: S (nF x nF) and b.  camera_terms = 0 leaves out the FrameDistance / CameraStabilization
  // rows, giving one landmark shard's contribution to the multi-GPU all-reduce.
  bool ReducedSystem(double radius, bool camera_terms, double* S_out, double* b_out);

  const std::vector<double>& scale() const { return scale_; }
  int nF() const { return nF_; }
  int nE() const { return nE_; }

 private:
  sg_problem* p_;
  Options opt_;
  Cauchy cauchy_, dist_cauchy_, stab_cauchy_;
  // Layout of the local parameter vector: camera side [0,nF) then points [nF, nF+nE).
  std::vector<int> rot_col_, trans_col_, k_col_, pt_col_;
  int nF_ = 0, nE_ = 0;
  std::vector<char> obs_fixed_;                 // all parameter blocks constant -> fixed cost
  std::vector<std::vector<int>> point_obs_;     // free point -> variable obs
  std::vector<int> var_obs_;
  std::vector<double> scale_;
  double fixed_cost_ = 0.0;

  // Linearization (scaled after the first evaluation).
  std::vector<ObsLin> lin_;
  std::vector<double> dist_r_, dist_J_;         // per FD: r, J (6: d/dt_a, d/dt_b)
  std::vector<double> stab_r_, stab_J_;         // per camera: 7 r, 7x7 J
  std::vector<double> gradient_;

  void Layout();
  int Threads() const { return std::max(1, opt_.nthreads); }

  // State vectors (global params) for the free blocks.
  struct State { std::vector<double> q, t, X, k; };
  State Capture() const {
    State s;
    s.q.assign(p_->q, p_->q + 4 * p_->num_frames);
    s.t.assign(p_->t, p_->t + 3 * p_->num_frames);
    s.X.assign(p_->X, p_->X + 4 * p_->num_points);
    s.k.assign(p_->k, p_->k + 7 * p_->num_cameras);
    return s;
  }
  double NormSq(const State& s) const;
  double DiffNormSq(const State& a, const State& b) const;

  bool EvalObs(const State& s, int o, bool jac, ObsLin* L) const;
  bool Evaluate(const State& s, bool jac, double* cost);
  void ScaleJacobian();
  void SquaredColumnNorm(std::vector<double>* d) const;
  bool SolveLinear(const std::vector<double>& D2, std::vector<double>* x);
  double ModelCostChange(const std::vector<double>& step) const;
  void Plus(const State& s, const std::vector<double>& delta, State* out) const;
  void Store(const State& s);

  // ReducedSystem capture: when set, SolveLinear stops after assembling S and b.
  double* cap_S_ = nullptr;
  double* cap_b_ = nullptr;
  bool cap_camera_terms_ = true;
};

void Solver::Layout() {
  const sg_problem& p = *p_;
  rot_col_.assign(p.num_frames, -1);
  trans_col_.assign(p.num_frames, -1);
  k_col_.assign(p.num_cameras, -1);
  pt_col_.assign(p.num_points, -1);
  int c = 0;
  for (int f = 0; f < p.num_frames; ++f) {
    if (p.frame_rot_free[f]) { rot_col_[f] = c; c += 3; }
    if (p.frame_trans_free[f]) { trans_col_[f] = c; c += 3; }
  }
  if (p.cameras_free)
    for (int i = 0; i < p.num_cameras; ++i) { k_col_[i] = c; c += 7; }
  nF_ = c;
  int e = 0;
  for (int i = 0; i < p.num_points; ++i)
    if (p.point_free[i]) { pt_col_[i] = nF_ + e; e += 4; }
  nE_ = e;
  obs_fixed_.assign(p.num_obs, 0);
  point_obs_.assign(p.num_points, {});
  var_obs_.clear();
  for (int o = 0; o < p.num_obs; ++o) {
    const int f = p.obs_frame[o], pt = p.obs_point[o];
    const bool any_free = rot_col_[f] >= 0 || trans_col_[f] >= 0 || pt_col_[pt] >= 0 ||
                          k_col_[p.frame_camera[f]] >= 0;
    obs_fixed_[o] = !any_free;
    if (any_free) {
      var_obs_.push_back(o);
      if (pt_col_[pt] >= 0) point_obs_[pt].push_back(o);
    }
  }
  lin_.assign(p.num_obs, ObsLin());
  dist_r_.assign(p.num_dist, 0.0);
  dist_J_.assign(6 * p.num_dist, 0.0);
  stab_r_.assign(7 * p.num_cameras, 0.0);
  stab_J_.assign(49 * p.num_cameras, 0.0);
}

double Solver::NormSq(const State& s) const {
  const sg_problem& p = *p_;
  double n = 0.0;
  for (int f = 0; f < p.num_frames; ++f) {
    if (rot_col_[f] >= 0) for (int j = 0; j < 4; ++j) n += s.q[4 * f + j] * s.q[4 * f + j];
    if (trans_col_[f] >= 0) for (int j = 0; j < 3; ++j) n += s.t[3 * f + j] * s.t[3 * f + j];
  }
  for (int c = 0; c < p.num_cameras; ++c)
    if (k_col_[c] >= 0) for (int j = 0; j < 7; ++j) n += s.k[7 * c + j] * s.k[7 * c + j];
  for (int i = 0; i < p.num_points; ++i)
    if (pt_col_[i] >= 0) for (int j = 0; j < 4; ++j) n += s.X[4 * i + j] * s.X[4 * i + j];
  return n;
}

double Solver::DiffNormSq(const State& a, const State& b) const {
  const sg_problem& p = *p_;
  double n = 0.0;
  auto sq = [](double x) { return x * x; };
  for (int f = 0; f < p.num_frames; ++f) {
    if (rot_col_[f] >= 0) for (int j = 0; j < 4; ++j) n += sq(a.q[4 * f + j] - b.q[4 * f + j]);
    if (trans_col_[f] >= 0) for (int j = 0; j < 3; ++j) n += sq(a.t[3 * f + j] - b.t[3 * f + j]);
  }
  for (int c = 0; c < p.num_cameras; ++c)
    if (k_col_[c] >= 0) for (int j = 0; j < 7; ++j) n += sq(a.k[7 * c + j] - b.k[7 * c + j]);
  for (int i = 0; i < p.num_points; ++i)
    if (pt_col_[i] >= 0) for (int j = 0; j < 4; ++j) n += sq(a.X[4 * i + j] - b.X[4 * i + j]);
  return n;
}

// One ReprojectionError residual block (slam.cpp:60-84) through AutoDiff (Jet<18> over q,t,k,X),
// CauchyLoss + corrector, and the quaternion local parameterization.
bool Solver::EvalObs(const State& s, int o, bool jac, ObsLin* L) const {
  const sg_problem& p = *p_;
  const int f = p.obs_frame[o], pt = p.obs_point[o], cam = p.frame_camera[f];
  const double* q = &s.q[4 * f];
  const double* t = &s.t[3 * f];
  const double* k = &s.k[7 * cam];
  const double* X = &s.X[4 * pt];
  double r[2];
  double J[2][18];
  if (jac) {
    typedef Jet<18> J18;
    J18 jq[4], jt[3], jk[7], jX[4], out[2];
    for (int i = 0; i < 4; ++i) jq[i] = J18(q[i], i);
    for (int i = 0; i < 3; ++i) jt[i] = J18(t[i], 4 + i);
    for (int i = 0; i < 7; ++i) jk[i] = J18(k[i], 7 + i);
    for (int i = 0; i < 4; ++i) jX[i] = J18(X[i], 14 + i);
    if (!ProjectPoint(jq, jt, jk, jX, out)) return false;
    r[0] = out[0].a - p.obs_pt[2 * o];
    r[1] = out[1].a - p.obs_pt[2 * o + 1];
    for (int i = 0; i < 2; ++i) for (int j = 0; j < 18; ++j) J[i][j] = out[i].v[j];
  } else {
    double out[2];
    if (!ProjectPoint(q, t, k, X, out)) return false;
    r[0] = out[0] - p.obs_pt[2 * o];
    r[1] = out[1] - p.obs_pt[2 * o + 1];
  }
  const double sq = r[0] * r[0] + r[1] * r[1];
  double rho[3];
  cauchy_.Evaluate(sq, rho);
  L->cost = 0.5 * rho[0];
  const double sr = std::sqrt(rho[1]);
  L->r[0] = sr * r[0];
  L->r[1] = sr * r[1];
  if (jac) {
    double Lq[12];
    QuatLocalJacobian(q, Lq);
    for (int i = 0; i < 2; ++i) {
      for (int c = 0; c < 3; ++c) {
        double acc = 0.0;
        for (int g = 0; g < 4; ++g) acc += J[i][g] * Lq[3 * g + c];
        L->Jc[i][c] = sr * acc;
      }
      for (int c = 0; c < 3; ++c) L->Jc[i][3 + c] = sr * J[i][4 + c];
      for (int c = 0; c < 7; ++c) L->Jc[i][6 + c] = sr * J[i][7 + c];
      for (int c = 0; c < 4; ++c) L->Jp[i][c] = sr * J[i][14 + c];
    }
  }
  return true;
}

bool Solver::Evaluate(const State& s, bool jac, double* cost) {
  const sg_problem& p = *p_;
  const int nv = (int)var_obs_.size();
  const int nt = Threads();
  std::vector<double> part(nt, 0.0);
  std::vector<int> fail(nt, 0);
#pragma omp parallel num_threads(nt)
  {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    const int lo = (int)((long long)nv * tid / nt), hi = (int)((long long)nv * (tid + 1) / nt);
    double acc = 0.0;
    int bad = 0;
    ObsLin tmp;
    for (int i = lo; i < hi; ++i) {
      const int o = var_obs_[i];
      ObsLin* L = jac ? &lin_[o] : &tmp;
      if (!EvalObs(s, o, jac, L)) { bad = 1; continue; }
      acc += L->cost;
    }
    part[tid] = acc;
    fail[tid] = bad;
  }
  double c = 0.0;
  for (int i = 0; i < nt; ++i) { c += part[i]; if (fail[i]) return false; }
  // FrameDistance (slam.cpp:86-105): r = 0.1 (|t_a - t_b| - 150), CauchyLoss(15).
  for (int d = 0; d < p.num_dist; ++d) {
    const double* ta = &s.t[3 * p.dist_frame[d]];
    const double* tb = &s.t[3 * p.dist_prev[d]];
    const double e0 = ta[0] - tb[0], e1 = ta[1] - tb[1], e2 = ta[2] - tb[2];
    const double dist = std::sqrt(e0 * e0 + e1 * e1 + e2 * e2);
    const double r = 0.1 * (dist - p.dist_target);
    double rho[3];
    dist_cauchy_.Evaluate(r * r, rho);
    c += 0.5 * rho[0];
    if (jac) {
      const double sr = std::sqrt(rho[1]);
      dist_r_[d] = sr * r;
      const double g = 0.1 / dist;
      const double ga[3] = {g * e0, g * e1, g * e2};
      for (int j = 0; j < 3; ++j) {
        dist_J_[6 * d + j] = trans_col_[p.dist_frame[d]] >= 0 ? sr * ga[j] : 0.0;
        dist_J_[6 * d + 3 + j] = trans_col_[p.dist_prev[d]] >= 0 ? -sr * ga[j] : 0.0;
      }
    }
  }
  // CameraStabilization (slam.cpp:107-124) with CauchyLoss(5) when the intrinsics are free.
  if (p.cameras_free) {
    for (int cam = 0; cam < p.num_cameras; ++cam) {
      typedef Jet<7> J7;
      J7 kk[7];
      for (int i = 0; i < 7; ++i) kk[i] = J7(s.k[7 * cam + i], i);
      J7 res[7];
      res[0] = 1000.0 * kk[0] * kk[0];
      res[1] = 1000.0 * kk[1] * kk[1];
      res[2] = 1000.0 * kk[2] * kk[2];
      res[3] = 0.1 * (kk[3] - 416.0) * (kk[3] - 416.0);
      res[4] = 0.1 * (kk[4] + kk[3]) * (kk[4] + kk[3]);
      res[5] = 0.01 * (kk[5] - 320.0) * (kk[5] - 320.0);
      res[6] = 0.01 * (kk[6] - 240.0) * (kk[6] - 240.0);
      double sq = 0.0;
      for (int i = 0; i < 7; ++i) sq += res[i].a * res[i].a;
      double rho[3];
      stab_cauchy_.Evaluate(sq, rho);
      c += 0.5 * rho[0];
      if (jac) {
        const double sr = std::sqrt(rho[1]);
        for (int i = 0; i < 7; ++i) {
          stab_r_[7 * cam + i] = sr * res[i].a;
          for (int j = 0; j < 7; ++j) stab_J_[49 * cam + 7 * i + j] = sr * res[i].v[j];
        }
      }
    }
  }
  if (jac) {
    // Gradient g = J^T r (unscaled, local).
    gradient_.assign(nF_ + nE_, 0.0);
    for (int o : var_obs_) {
      const ObsLin& L = lin_[o];
      const int f = p.obs_frame[o], pt = p.obs_point[o], cam = p.frame_camera[f];
      for (int i = 0; i < 2; ++i) {
        if (rot_col_[f] >= 0) for (int c2 = 0; c2 < 3; ++c2) gradient_[rot_col_[f] + c2] += L.Jc[i][c2] * L.r[i];
        if (trans_col_[f] >= 0) for (int c2 = 0; c2 < 3; ++c2) gradient_[trans_col_[f] + c2] += L.Jc[i][3 + c2] * L.r[i];
        if (k_col_[cam] >= 0) for (int c2 = 0; c2 < 7; ++c2) gradient_[k_col_[cam] + c2] += L.Jc[i][6 + c2] * L.r[i];
        if (pt_col_[pt] >= 0) for (int c2 = 0; c2 < 4; ++c2) gradient_[pt_col_[pt] + c2] += L.Jp[i][c2] * L.r[i];
      }
    }
    for (int d = 0; d < p.num_dist; ++d) {
      const int a = trans_col_[p.dist_frame[d]], b = trans_col_[p.dist_prev[d]];
      for (int j = 0; j < 3; ++j) {
        if (a >= 0) gradient_[a + j] += dist_J_[6 * d + j] * dist_r_[d];
        if (b >= 0) gradient_[b + j] += dist_J_[6 * d + 3 + j] * dist_r_[d];
      }
    }
    if (p.cameras_free)
      for (int cam = 0; cam < p.num_cameras; ++cam)
        for (int i = 0; i < 7; ++i)
          for (int j = 0; j < 7; ++j)
            gradient_[k_col_[cam] + j] += stab_J_[49 * cam + 7 * i + j] * stab_r_[7 * cam + i];
  }
  *cost = c;
  return true;
}

// Squared column norms of the (current, possibly scaled) Jacobian.
void Solver::SquaredColumnNorm(std::vector<double>* d) const {
  const sg_problem& p = *p_;
  d->assign(nF_ + nE_, 0.0);
  std::vector<double>& D = *d;
  for (int o : var_obs_) {
    const ObsLin& L = lin_[o];
    const int f = p.obs_frame[o], pt = p.obs_point[o], cam = p.frame_camera[f];
    for (int i = 0; i < 2; ++i) {
      if (rot_col_[f] >= 0) for (int c = 0; c < 3; ++c) D[rot_col_[f] + c] += L.Jc[i][c] * L.Jc[i][c];
      if (trans_col_[f] >= 0) for (int c = 0; c < 3; ++c) D[trans_col_[f] + c] += L.Jc[i][3 + c] * L.Jc[i][3 + c];
      if (k_col_[cam] >= 0) for (int c = 0; c < 7; ++c) D[k_col_[cam] + c] += L.Jc[i][6 + c] * L.Jc[i][6 + c];
      if (pt_col_[pt] >= 0) for (int c = 0; c < 4; ++c) D[pt_col_[pt] + c] += L.Jp[i][c] * L.Jp[i][c];
    }
  }
  for (int d2 = 0; d2 < p.num_dist; ++d2) {
    const int a = trans_col_[p.dist_frame[d2]], b = trans_col_[p.dist_prev[d2]];
    for (int j = 0; j < 3; ++j) {
      if (a >= 0) D[a + j] += dist_J_[6 * d2 + j] * dist_J_[6 * d2 + j];
      if (b >= 0) D[b + j] += dist_J_[6 * d2 + 3 + j] * dist_J_[6 * d2 + 3 + j];
    }
  }
  if (p.cameras_free)
    for (int cam = 0; cam < p.num_cameras; ++cam)
      for (int i = 0; i < 7; ++i)
        for (int j = 0; j < 7; ++j) D[k_col_[cam] + j] += stab_J_[49 * cam + 7 * i + j] * stab_J_[49 * cam + 7 * i + j];
}

void Solver::ScaleJacobian() {
  const sg_problem& p = *p_;
  for (int o : var_obs_) {
    ObsLin& L = lin_[o];
    const int f = p.obs_frame[o], pt = p.obs_point[o], cam = p.frame_camera[f];
    for (int i = 0; i < 2; ++i) {
      for (int c = 0; c < 3; ++c) L.Jc[i][c] *= rot_col_[f] >= 0 ? scale_[rot_col_[f] + c] : 0.0;
      for (int c = 0; c < 3; ++c) L.Jc[i][3 + c] *= trans_col_[f] >= 0 ? scale_[trans_col_[f] + c] : 0.0;
      for (int c = 0; c < 7; ++c) L.Jc[i][6 + c] *= k_col_[cam] >= 0 ? scale_[k_col_[cam] + c] : 0.0;
      for (int c = 0; c < 4; ++c) L.Jp[i][c] *= pt_col_[pt] >= 0 ? scale_[pt_col_[pt] + c] : 0.0;
    }
  }
  for (int d = 0; d < p.num_dist; ++d) {
    const int a = trans_col_[p.dist_frame[d]], b = trans_col_[p.dist_prev[d]];
    for (int j = 0; j < 3; ++j) {
      dist_J_[6 * d + j] *= a >= 0 ? scale_[a + j] : 0.0;
      dist_J_[6 * d + 3 + j] *= b >= 0 ? scale_[b + j] : 0.0;
    }
  }
  if (p.cameras_free)
    for (int cam = 0; cam < p.num_cameras; ++cam)
      for (int i = 0; i < 7; ++i)
        for (int j = 0; j < 7; ++j) stab_J_[49 * cam + 7 * i + j] *= scale_[k_col_[cam] + j];
}

// Dense LL^T in place (row-major, lower). Returns false on a non-positive (or NaN) pivot.
static bool Cholesky(std::vector<double>& A, int n) {
  for (int j = 0; j < n; ++j) {
    double d = A[(size_t)j * n + j];
    for (int k = 0; k < j; ++k) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
    if (!(d > 0.0)) return false;
    const double ljj = std::sqrt(d);
    A[(size_t)j * n + j] = ljj;
    const double inv = 1.0 / ljj;
    for (int i = j + 1; i < n; ++i) {
      double s = A[(size_t)i * n + j];
      const double* ri = &A[(size_t)i * n];
      const double* rj = &A[(size_t)j * n];
      for (int k = 0; k < j; ++k) s -= ri[k] * rj[k];
      A[(size_t)i * n + j] = s * inv;
    }
  }
  return true;
}
static void CholSolve(const std::vector<double>& L, int n, double* b) {
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= L[(size_t)i * n + k] * b[k];
    b[i] = s / L[(size_t)i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int k = i + 1; k < n; ++k) s -= L[(size_t)k * n + i] * b[k];
    b[i] = s / L[(size_t)i * n + i];
  }
}
// 4x4 SPD inverse via LL^T (Eigen llt().solve(Identity) in the Schur eliminator).
static bool Inverse4(const double* A, double* Ainv) {
  std::vector<double> L(A, A + 16);
  if (!Cholesky(L, 4)) return false;
  for (int c = 0; c < 4; ++c) {
    double e[4] = {0, 0, 0, 0};
    e[c] = 1.0;
    CholSolve(L, 4, e);
    for (int r = 0; r < 4; ++r) Ainv[4 * r + c] = e[r];
  }
  return true;
}

// Solve (A^T A + D^2) x = A^T b by Schur elimination of the point blocks (SPARSE_SCHUR).
bool Solver::SolveLinear(const std::vector<double>& D2, std::vector<double>* xout) {
  const sg_problem& p = *p_;
  const int n = nF_;
  std::vector<double>& x = *xout;
  x.assign(nF_ + nE_, 0.0);
  const int nt = Threads();
  std::vector<std::vector<double>> Sp(nt, std::vector<double>((size_t)n * n, 0.0));
  std::vector<std::vector<double>> bp(nt, std::vector<double>(n, 0.0));
  // Per-point eliminated data: V^-1 (16), g_e (4).
  std::vector<double> Vinv(16 * (size_t)p.num_points, 0.0), ge(4 * (size_t)p.num_points, 0.0);
  std::vector<char> ok_pt(p.num_points, 1);

  auto cols_of = [&](int o, int* cols) {
    const int f = p.obs_frame[o], cam = p.frame_camera[f];
    for (int c = 0; c < 3; ++c) cols[c] = rot_col_[f] >= 0 ? rot_col_[f] + c : -1;
    for (int c = 0; c < 3; ++c) cols[3 + c] = trans_col_[f] >= 0 ? trans_col_[f] + c : -1;
    for (int c = 0; c < 7; ++c) cols[6 + c] = k_col_[cam] >= 0 ? k_col_[cam] + c : -1;
  };

#pragma omp parallel num_threads(nt)
  {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    std::vector<double>& S = Sp[tid];
    std::vector<double>& b = bp[tid];
    // (1) camera-side normal equations F^T F, F^T b over every variable residual.
    const int nv = (int)var_obs_.size();
    const int lo = (int)((long long)nv * tid / nt), hi = (int)((long long)nv * (tid + 1) / nt);
    for (int i = lo; i < hi; ++i) {
      const int o = var_obs_[i];
      const ObsLin& L = lin_[o];
      int cols[13];
      cols_of(o, cols);
      for (int a = 0; a < 13; ++a) {
        if (cols[a] < 0) continue;
        b[cols[a]] += L.Jc[0][a] * L.r[0] + L.Jc[1][a] * L.r[1];
        for (int c = 0; c < 13; ++c) {
          if (cols[c] < 0) continue;
          S[(size_t)cols[a] * n + cols[c]] += L.Jc[0][a] * L.Jc[0][c] + L.Jc[1][a] * L.Jc[1][c];
        }
      }
    }
    // (2) eliminate each free point block.
    const int np = p.num_points;
    const int plo = (int)((long long)np * tid / nt), phi = (int)((long long)np * (tid + 1) / nt);
    std::vector<double> Y;
    for (int pt = plo; pt < phi; ++pt) {
      if (pt_col_[pt] < 0) continue;
      const std::vector<int>& ol = point_obs_[pt];
      double V[16] = {0}, g[4] = {0};
      for (int o : ol) {
        const ObsLin& L = lin_[o];
        for (int a = 0; a < 4; ++a) {
          g[a] += L.Jp[0][a] * L.r[0] + L.Jp[1][a] * L.r[1];
          for (int c = 0; c < 4; ++c) V[4 * a + c] += L.Jp[0][a] * L.Jp[0][c] + L.Jp[1][a] * L.Jp[1][c];
        }
      }
      for (int a = 0; a < 4; ++a) V[5 * a] += D2[pt_col_[pt] + a];
      double* Vi = &Vinv[16 * (size_t)pt];
      if (!Inverse4(V, Vi)) { ok_pt[pt] = 0; continue; }
      for (int a = 0; a < 4; ++a) ge[4 * (size_t)pt + a] = g[a];
      // W_o = F_o^T E_o (13x4);  Y_o = W_o V^-1.
      const int k = (int)ol.size();
      Y.assign((size_t)k * 52, 0.0);
      std::vector<double> W((size_t)k * 52, 0.0);
      for (int i = 0; i < k; ++i) {
        const ObsLin& L = lin_[ol[i]];
        for (int a = 0; a < 13; ++a)
          for (int c = 0; c < 4; ++c) W[52 * i + 4 * a + c] = L.Jc[0][a] * L.Jp[0][c] + L.Jc[1][a] * L.Jp[1][c];
        for (int a = 0; a < 13; ++a)
          for (int c = 0; c < 4; ++c) {
            double acc = 0.0;
            for (int m = 0; m < 4; ++m) acc += W[52 * i + 4 * a + m] * Vi[4 * m + c];
            Y[52 * i + 4 * a + c] = acc;
          }
      }
      for (int i = 0; i < k; ++i) {
        int ci[13];
        cols_of(ol[i], ci);
        for (int a = 0; a < 13; ++a) {
          if (ci[a] < 0) continue;
          double acc = 0.0;
          for (int m = 0; m < 4; ++m) acc += Y[52 * i + 4 * a + m] * g[m];
          b[ci[a]] -= acc;
        }
        for (int j = 0; j < k; ++j) {
          int cj[13];
          cols_of(ol[j], cj);
          for (int a = 0; a < 13; ++a) {
            if (ci[a] < 0) continue;
            for (int c = 0; c < 13; ++c) {
              if (cj[c] < 0) continue;
              double acc = 0.0;
              for (int m = 0; m < 4; ++m) acc += Y[52 * i + 4 * a + m] * W[52 * j + 4 * c + m];
              S[(size_t)ci[a] * n + cj[c]] -= acc;
            }
          }
        }
      }
    }
  }
  for (int pt = 0; pt < p.num_points; ++pt)
    if (!ok_pt[pt]) return false;
  std::vector<double> S((size_t)n * n, 0.0), b(n, 0.0);
  for (int tid = 0; tid < nt; ++tid) {
    for (size_t i = 0; i < S.size(); ++i) S[i] += Sp[tid][i];
    for (int i = 0; i < n; ++i) b[i] += bp[tid][i];
  }
  // FrameDistance / CameraStabilization rows (no point block).
  const bool camera_terms = cap_S_ == nullptr || cap_camera_terms_;
  for (int d = 0; d < (camera_terms ? p.num_dist : 0); ++d) {
    int cols[6];
    for (int j = 0; j < 3; ++j) {
      cols[j] = trans_col_[p.dist_frame[d]] >= 0 ? trans_col_[p.dist_frame[d]] + j : -1;
      cols[3 + j] = trans_col_[p.dist_prev[d]] >= 0 ? trans_col_[p.dist_prev[d]] + j : -1;
    }
    const double* J = &dist_J_[6 * d];
    for (int a = 0; a < 6; ++a) {
      if (cols[a] < 0) continue;
      b[cols[a]] += J[a] * dist_r_[d];
      for (int c = 0; c < 6; ++c)
        if (cols[c] >= 0) S[(size_t)cols[a] * n + cols[c]] += J[a] * J[c];
    }
  }
  if (p.cameras_free && camera_terms)
    for (int cam = 0; cam < p.num_cameras; ++cam) {
      const int c0 = k_col_[cam];
      for (int i = 0; i < 7; ++i) {
        const double* Jr = &stab_J_[49 * cam + 7 * i];
        for (int a = 0; a < 7; ++a) {
          b[c0 + a] += Jr[a] * stab_r_[7 * cam + i];
          for (int c = 0; c < 7; ++c) S[(size_t)(c0 + a) * n + c0 + c] += Jr[a] * Jr[c];
        }
      }
    }
  if (cap_S_) {
    std::copy(S.begin(), S.end(), cap_S_);
    std::copy(b.begin(), b.end(), cap_b_);
    return false;
  }
  for (int i = 0; i < n; ++i) S[(size_t)i * n + i] += D2[i];
  if (!Cholesky(S, n)) return false;
  CholSolve(S, n, b.data());
  for (int i = 0; i < n; ++i) x[i] = b[i];
  // Back-substitute the points: x_e = V^-1 (g_e - E^T F x_F).
  for (int pt = 0; pt < p.num_points; ++pt) {
    if (pt_col_[pt] < 0) continue;
    double rhs[4];
    for (int a = 0; a < 4; ++a) rhs[a] = ge[4 * (size_t)pt + a];
    for (int o : point_obs_[pt]) {
      const ObsLin& L = lin_[o];
      int cols[13];
      cols_of(o, cols);
      double fx[2] = {0.0, 0.0};
      for (int a = 0; a < 13; ++a)
        if (cols[a] >= 0) { fx[0] += L.Jc[0][a] * x[cols[a]]; fx[1] += L.Jc[1][a] * x[cols[a]]; }
      for (int a = 0; a < 4; ++a) rhs[a] -= L.Jp[0][a] * fx[0] + L.Jp[1][a] * fx[1];
    }
    const double* Vi = &Vinv[16 * (size_t)pt];
    for (int a = 0; a < 4; ++a) {
      double acc = 0.0;
      for (int c = 0; c < 4; ++c) acc += Vi[4 * a + c] * rhs[c];
      x[pt_col_[pt] + a] = acc;
    }
  }
  for (double v : x)
    if (!std::isfinite(v)) return false;
  return true;
}

bool Solver::ReducedSystem(double radius, bool camera_terms, double* S_out, double* b_out) {
  State x = Capture();
  double cost = 0.0;
  if (!Evaluate(x, true, &cost)) return false;
  std::vector<double> diag, D2(nF_ + nE_, 0.0), xs;
  SquaredColumnNorm(&diag);
  for (int i = nF_; i < nF_ + nE_; ++i)
    D2[i] = std::min(std::max(diag[i], opt_.o.min_lm_diagonal), opt_.o.max_lm_diagonal) / radius;
  cap_S_ = S_out;
  cap_b_ = b_out;
  cap_camera_terms_ = camera_terms;
  SolveLinear(D2, &xs);
  cap_S_ = cap_b_ = nullptr;
  return true;
}

// -(J s) . (r + (J s)/2) with the scaled, corrected Jacobian.
double Solver::ModelCostChange(const std::vector<double>& s) const {
  const sg_problem& p = *p_;
  double mc = 0.0;
  for (int o : var_obs_) {
    const ObsLin& L = lin_[o];
    const int f = p.obs_frame[o], pt = p.obs_point[o], cam = p.frame_camera[f];
    double m[2] = {0.0, 0.0};
    for (int i = 0; i < 2; ++i) {
      if (rot_col_[f] >= 0) for (int c = 0; c < 3; ++c) m[i] += L.Jc[i][c] * s[rot_col_[f] + c];
      if (trans_col_[f] >= 0) for (int c = 0; c < 3; ++c) m[i] += L.Jc[i][3 + c] * s[trans_col_[f] + c];
      if (k_col_[cam] >= 0) for (int c = 0; c < 7; ++c) m[i] += L.Jc[i][6 + c] * s[k_col_[cam] + c];
      if (pt_col_[pt] >= 0) for (int c = 0; c < 4; ++c) m[i] += L.Jp[i][c] * s[pt_col_[pt] + c];
    }
    mc -= m[0] * (L.r[0] + 0.5 * m[0]) + m[1] * (L.r[1] + 0.5 * m[1]);
  }
  for (int d = 0; d < p.num_dist; ++d) {
    const int a = trans_col_[p.dist_frame[d]], b = trans_col_[p.dist_prev[d]];
    double m = 0.0;
    for (int j = 0; j < 3; ++j) {
      if (a >= 0) m += dist_J_[6 * d + j] * s[a + j];
      if (b >= 0) m += dist_J_[6 * d + 3 + j] * s[b + j];
    }
    mc -= m * (dist_r_[d] + 0.5 * m);
  }
  if (p.cameras_free)
    for (int cam = 0; cam < p.num_cameras; ++cam)
      for (int i = 0; i < 7; ++i) {
        double m = 0.0;
        for (int j = 0; j < 7; ++j) m += stab_J_[49 * cam + 7 * i + j] * s[k_col_[cam] + j];
        mc -= m * (stab_r_[7 * cam + i] + 0.5 * m);
      }
  return mc;
}

void Solver::Plus(const State& s, const std::vector<double>& delta, State* out) const {
  const sg_problem& p = *p_;
  *out = s;
  for (int f = 0; f < p.num_frames; ++f) {
    if (rot_col_[f] >= 0) QuatPlus(&s.q[4 * f], &delta[rot_col_[f]], &out->q[4 * f]);
    if (trans_col_[f] >= 0) for (int j = 0; j < 3; ++j) out->t[3 * f + j] = s.t[3 * f + j] + delta[trans_col_[f] + j];
  }
  for (int c = 0; c < p.num_cameras; ++c)
    if (k_col_[c] >= 0) for (int j = 0; j < 7; ++j) out->k[7 * c + j] = s.k[7 * c + j] + delta[k_col_[c] + j];
  for (int i = 0; i < p.num_points; ++i)
    if (pt_col_[i] >= 0) for (int j = 0; j < 4; ++j) out->X[4 * i + j] = s.X[4 * i + j] + delta[pt_col_[i] + j];
}

void Solver::Store(const State& s) {
  std::copy(s.q.begin(), s.q.end(), p_->q);
  std::copy(s.t.begin(), s.t.end(), p_->t);
  std::copy(s.X.begin(), s.X.end(), p_->X);
  std::copy(s.k.begin(), s.k.end(), p_->k);
}

void Solver::Solve(sg_solver_summary* sum) {
  const sg_solver_options& o = opt_.o;
  std::memset(sum, 0, sizeof(*sum));
  sum->termination_type = SG_DID_NOT_RUN;
  State x = Capture();
  // Fixed cost: residual blocks whose parameter blocks are all constant (Program::RemoveFixedBlocks).
  fixed_cost_ = 0.0;
  for (int ob = 0; ob < p_->num_obs; ++ob) {
    if (!obs_fixed_[ob]) continue;
    ObsLin L;
    if (!EvalObs(x, ob, false, &L)) {
      sum->ok = 0; sum->termination_type = SG_DID_NOT_RUN; return;  // evaluation failed during removal
    }
    fixed_cost_ += L.cost;
  }
  sum->fixed_cost = fixed_cost_;
  if (nF_ + nE_ == 0) {  // no free parameter blocks: nothing to do, not an error
    sum->ok = 1; sum->termination_type = SG_FUNCTION_TOLERANCE;
    sum->initial_cost = sum->final_cost = fixed_cost_;
    return;
  }
  double cost = 0.0;
  if (!Evaluate(x, true, &cost)) {
    sum->ok = 0; sum->termination_type = SG_NUMERICAL_FAILURE; return;
  }
  sum->initial_cost = cost + fixed_cost_;
  // summary.final_cost = min over the pushed iteration summaries (SetSummaryFinalCost); the terminating
  // iteration is not pushed (Ceres 1.8 returns before push_back).
  double pushed_min_cost = cost;
  // Jacobi scaling: scale = 1 / (1 + sqrt(colnorm^2)), computed once.
  scale_.assign(nF_ + nE_, 1.0);
  if (o.jacobi_scaling) {
    SquaredColumnNorm(&scale_);
    for (double& v : scale_) v = 1.0 / (1.0 + std::sqrt(v));
    ScaleJacobian();
  }
  double gmax = 0.0;
  for (double g : gradient_) gmax = std::max(gmax, std::fabs(g));
  const double abs_gtol = o.gradient_tolerance * gmax;
  int num_iterations = 1;  // iteration 0 pushed
  if (gmax <= abs_gtol) {
    sum->termination_type = SG_GRADIENT_TOLERANCE; sum->ok = 1; sum->num_iterations = 1;
    sum->final_cost = cost + fixed_cost_; return;
  }
  double x_norm = std::sqrt(NormSq(x));
  // LevenbergMarquardtStrategy state.
  double radius = o.initial_trust_region_radius, decrease_factor = 2.0;
  bool reuse_diagonal = false;
  std::vector<double> diagonal, D2(nF_ + nE_), xsol, step(nF_ + nE_), delta(nF_ + nE_);
  int consecutive_invalid = 0;
  int lm_iters = 0;
  State xc;
  sum->ok = 1;
  while (true) {
    if (!o.disable_termination && num_iterations - 1 >= o.max_num_iterations) {
      sum->termination_type = SG_NO_CONVERGENCE; break;
    }
    if (o.disable_termination && lm_iters >= o.max_num_iterations) { sum->termination_type = SG_NO_CONVERGENCE; break; }
    ++lm_iters;
    // ComputeStep.
    if (!reuse_diagonal) {
      SquaredColumnNorm(&diagonal);
      for (double& v : diagonal) v = std::min(std::max(v, o.min_lm_diagonal), o.max_lm_diagonal);
    }
    for (size_t i = 0; i < D2.size(); ++i) D2[i] = diagonal[i] / radius;
    bool valid = SolveLinear(D2, &xsol);
    if (getenv("ORACLE_DEBUG")) fprintf(stderr, "it %d radius %g solve %d\n", lm_iters, radius, (int)valid);
    reuse_diagonal = true;
    double model_cost_change = 0.0;
    if (valid) {
      for (size_t i = 0; i < step.size(); ++i) step[i] = -xsol[i];
      model_cost_change = ModelCostChange(step);
      if (model_cost_change < 0.0) valid = false;
      if (getenv("ORACLE_DEBUG")) fprintf(stderr, "   mcc %g cost %g\n", model_cost_change, cost);
    }
    bool successful = false;
    double relative_decrease = 0.0;
    if (!valid) {
      ++sum->num_invalid_steps;
      if (++consecutive_invalid >= o.max_num_consecutive_invalid_steps && !o.disable_termination) {
        sum->termination_type = SG_NUMERICAL_FAILURE; sum->ok = 0; break;
      }
    } else {
      consecutive_invalid = 0;
      for (size_t i = 0; i < step.size(); ++i) delta[i] = step[i] * scale_[i];
      Plus(x, delta, &xc);
      double new_cost = std::numeric_limits<double>::max();
      if (!Evaluate(xc, false, &new_cost)) new_cost = std::numeric_limits<double>::max();
      const double step_norm = std::sqrt(DiffNormSq(x, xc));
      if (!o.disable_termination &&
          step_norm <= o.parameter_tolerance * (x_norm + o.parameter_tolerance)) {
        sum->termination_type = SG_PARAMETER_TOLERANCE; break;
      }
      const double cost_change = cost - new_cost;
      if (!o.disable_termination && std::fabs(cost_change) < o.function_tolerance * cost) {
        sum->termination_type = SG_FUNCTION_TOLERANCE; break;
      }
      relative_decrease = cost_change / model_cost_change;
      successful = relative_decrease > o.min_relative_decrease;
    }
    if (successful) {
      ++sum->num_successful_steps;
      radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * relative_decrease - 1.0, 3));
      radius = std::min(o.max_trust_region_radius, radius);
      decrease_factor = 2.0;
      reuse_diagonal = false;
      x = xc;
      x_norm = std::sqrt(NormSq(x));
      if (!Evaluate(x, true, &cost)) { sum->termination_type = SG_NUMERICAL_FAILURE; sum->ok = 0; break; }
      if (o.jacobi_scaling) ScaleJacobian();
      double g2 = 0.0;
      for (double g : gradient_) g2 = std::max(g2, std::fabs(g));
      if (!o.disable_termination && g2 <= abs_gtol) { sum->termination_type = SG_GRADIENT_TOLERANCE; break; }
    } else {
      ++sum->num_unsuccessful_steps;
      radius = radius / decrease_factor;   // StepRejected / StepIsInvalid
      decrease_factor *= 2.0;
      reuse_diagonal = true;
    }
    if (!o.disable_termination && radius < o.min_trust_region_radius) {
      sum->termination_type = SG_PARAMETER_TOLERANCE; break;
    }
    ++num_iterations;
    pushed_min_cost = std::min(pushed_min_cost, cost);
  }
  sum->num_iterations = num_iterations;
  sum->num_lm_iterations = lm_iters;
  sum->final_cost = pushed_min_cost + fixed_cost_;
  sum->trust_region_radius = radius;
  Store(x);
}

bool Solver::EvaluateResiduals(double* r_out, double* cost_out, int* nfail) {
  const sg_problem& p = *p_;
  State s = Capture();
  double c = 0.0;
  int bad = 0;
  for (int o = 0; o < p.num_obs; ++o) {
    const int f = p.obs_frame[o], pt = p.obs_point[o], cam = p.frame_camera[f];
    double out[2];
    if (!ProjectPoint(&s.q[4 * f], &s.t[3 * f], &s.k[7 * cam], &s.X[4 * pt], out)) {
      ++bad;
      r_out[2 * o] = r_out[2 * o + 1] = 0.0;
      continue;
    }
    const double r0 = out[0] - p.obs_pt[2 * o], r1 = out[1] - p.obs_pt[2 * o + 1];
    r_out[2 * o] = r0;
    r_out[2 * o + 1] = r1;
    double rho[3];
    cauchy_.Evaluate(r0 * r0 + r1 * r1, rho);
    if (!obs_fixed_[o]) c += 0.5 * rho[0];
  }
  *cost_out = c;
  *nfail = bad;
  return bad == 0;
}

}  // namespace oracle

// ================================================================================================
// C API of the oracle (prefix or_).  Used only by tests/, smoke() and bench.py's cpu_baseline leg.
extern "C" {

struct or_problem {
  oracle::OwnedProblem owned;
};

void or_default_options(sg_solver_options* o) {
  o->max_num_iterations = 1000;
  o->function_tolerance = 1e-7;
  o->gradient_tolerance = 1e-10;
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
}

// Slam::SolveFrames frame selection (slam.cpp:417-434) + SetupProblem; returns a handle or NULL when the
// reference aborts (fewer than 2 used frames).
or_problem* or_problem_from_map_frames(const sg_map* m, int num_to_solve, int num_to_present, double range) {
  std::map<int, bool> frames;
  for (int i = 0; i < m->num_frames; ++i) {
    const int f = m->num_frames - i - 1;
    if (i < num_to_solve) frames[f] = false;
    else if (i < num_to_present) frames[f] = true;
    else break;
  }
  or_problem* h = new or_problem;
  if (!oracle::SetupProblem(*m, range, frames, false, &h->owned)) { delete h; return nullptr; }
  return h;
}

or_problem* or_problem_from_map_all(const sg_map* m, double range, int solve_cameras) {
  std::map<int, bool> frames;
  for (int f = 0; f < m->num_frames; ++f) frames[f] = false;
  or_problem* h = new or_problem;
  if (!oracle::SetupProblem(*m, range, frames, solve_cameras != 0, &h->owned)) { delete h; return nullptr; }
  return h;
}

sg_problem* or_problem_view(or_problem* h) { return &h->owned.p; }
void or_problem_free(or_problem* h) { delete h; }

// Solve a problem in place (p's q/t/X/k are updated).
int or_solve(sg_problem* p, const sg_solver_options* o, int nthreads, sg_solver_summary* s) {
  oracle::Options opt;
  opt.o = *o;
  opt.nthreads = nthreads;
  oracle::Solver solver(p, opt);
  solver.Solve(s);
  return 0;
}

// One landmark shard's (camera_terms = 0) or the whole problem's reduced camera system; returns its
// dimension n (S is n x n row-major) or -1 if the evaluation fails.  nmax bounds the output arrays.
int or_reduced_system(sg_problem* p, double radius, int camera_terms, int nthreads, double* S, double* b,
                      int nmax) {
  oracle::Options opt;
  or_default_options(&opt.o);
  opt.nthreads = nthreads;
  oracle::Solver solver(p, opt);
  if (solver.nF() > nmax) return -1;
  if (!solver.ReducedSystem(radius, camera_terms != 0, S, b)) return -1;
  return solver.nF();
}

// Corrected-free reprojection residuals (proj - pt) for every problem observation at the current state.
int or_evaluate(sg_problem* p, double* residuals, double* cost, int* nfail) {
  oracle::Options opt;
  or_default_options(&opt.o);
  opt.nthreads = 1;
  oracle::Solver solver(p, opt);
  solver.EvaluateResiduals(residuals, cost, nfail);
  return 0;
}

// Jacobian of one observation through AutoDiff (Jet<18>): out[2*18] d(uv)/d(q,t,k,X) global, and uv.
int or_project_jet(const double* q, const double* t, const double* k, const double* X, double* uv, double* J) {
  typedef oracle::Jet<18> J18;
  J18 jq[4], jt[3], jk[7], jX[4], out[2];
  for (int i = 0; i < 4; ++i) jq[i] = J18(q[i], i);
  for (int i = 0; i < 3; ++i) jt[i] = J18(t[i], 4 + i);
  for (int i = 0; i < 7; ++i) jk[i] = J18(k[i], 7 + i);
  for (int i = 0; i < 4; ++i) jX[i] = J18(X[i], 14 + i);
  if (!oracle::ProjectPoint(jq, jt, jk, jX, out)) return 0;
  uv[0] = out[0].a; uv[1] = out[1].a;
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 18; ++j) J[18 * i + j] = out[i].v[j];
  return 1;
}

// project.h on double for n points (known-answer tests). ok[i] = 0 on behind-camera rejection.
int or_project(int n, const double* q, const double* t, const double* k, const double* X, double* uv, int* ok) {
  for (int i = 0; i < n; ++i)
    ok[i] = oracle::ProjectPoint(q + 4 * i, t + 3 * i, k + 7 * i, X + 4 * i, uv + 2 * i) ? 1 : 0;
  return 0;
}

void or_quat_plus(const double* x, const double* d, double* out) { oracle::QuatPlus(x, d, out); }

// Slam::ReprojectMap (slam.cpp:523-548): every observation of every frame, disabled ones included.
// error = pt, then overwritten by proj - pt when the projection succeeds; running mean of |error|.
double or_reproject_map(sg_map* m) {
  double mean = 0.0, count = 0.0;
  for (int o = 0; o < m->num_obs; ++o) {
    const int f = m->obs_frame[o], pt = m->obs_point[o];
    m->obs_error[2 * o] = m->obs_pt[2 * o];
    m->obs_error[2 * o + 1] = m->obs_pt[2 * o + 1];
    double out[2];
    if (!oracle::ProjectPoint(&m->q[4 * f], &m->t[3 * f], &m->k[7 * m->frame_camera[f]], &m->X[4 * pt], out))
      continue;
    m->obs_error[2 * o] = out[0] - m->obs_pt[2 * o];
    m->obs_error[2 * o + 1] = out[1] - m->obs_pt[2 * o + 1];
    const double nrm = std::sqrt(m->obs_error[2 * o] * m->obs_error[2 * o] +
                                 m->obs_error[2 * o + 1] * m->obs_error[2 * o + 1]);
    mean = mean + (nrm - mean) / (count + 1);
    ++count;
  }
  return mean;
}

// Slam::SolveFrames / SolveAllFrames on a map (the map's blocks are updated in place).
// Returns 1 if solved (Run returned true), 0 otherwise; s receives the summary.
int or_slam_solve_frames(sg_map* m, int num_to_solve, int num_to_present, double range,
                         const sg_solver_options* o, int nthreads, sg_solver_summary* s) {
  std::memset(s, 0, sizeof(*s));
  or_problem* h = or_problem_from_map_frames(m, num_to_solve, num_to_present, range);
  if (!h) return 0;
  sg_problem* p = &h->owned.p;
  or_solve(p, o, nthreads, s);
  for (int f = 0; f < p->num_frames; ++f) {
    const int mf = p->frame_map_index[f];
    for (int j = 0; j < 4; ++j) m->q[4 * mf + j] = p->q[4 * f + j];
    for (int j = 0; j < 3; ++j) m->t[3 * mf + j] = p->t[3 * f + j];
  }
  for (int i = 0; i < p->num_points; ++i) {
    const int mp = p->point_map_index[i];
    for (int j = 0; j < 4; ++j) m->X[4 * mp + j] = p->X[4 * i + j];
  }
  or_problem_free(h);
  return s->ok;
}

int or_slam_solve_all_frames(sg_map* m, double range, int solve_cameras, const sg_solver_options* o,
                             int nthreads, sg_solver_summary* s) {
  std::memset(s, 0, sizeof(*s));
  or_problem* h = or_problem_from_map_all(m, range, solve_cameras);
  if (!h) return 0;
  sg_problem* p = &h->owned.p;
  sg_solver_options oo = *o;
  if (solve_cameras) oo.function_tolerance = 1e-9;  // Run(fine=true), slam.cpp:496-499
  or_solve(p, &oo, nthreads, s);
  for (int f = 0; f < p->num_frames; ++f) {
    const int mf = p->frame_map_index[f];
    for (int j = 0; j < 4; ++j) m->q[4 * mf + j] = p->q[4 * f + j];
    for (int j = 0; j < 3; ++j) m->t[3 * mf + j] = p->t[3 * f + j];
  }
  for (int i = 0; i < p->num_points; ++i) {
    const int mp = p->point_map_index[i];
    for (int j = 0; j < 4; ++j) m->X[4 * mp + j] = p->X[4 * i + j];
  }
  for (int i = 0; i < 7 * m->num_cameras; ++i) m->k[i] = p->k[i];
  or_problem_free(h);
  return s->ok;
}

}  // extern "C"
