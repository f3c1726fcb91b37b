// oracle_map.cpp — TEST INFRASTRUCTURE ONLY (the checker, never the product path).
//
// CPU restatement of the reference's LocalMap maintenance that runs on the BA residuals after every solve
// (main.cpp:584-605): LocalMap::Clean (localmap.cpp:283-398), LocalMap::ApplyEpipolarConstraint
// (localmap.cpp:232-276, EssentialMatrix 211-230), TrackedPoint::CheckFlags (localmap.cpp:44-83) and
// LocalMap::Normalize (localmap.cpp:114-155), on the sg_map structure-of-arrays view of a LocalMap.
//
// A point's observation list (TrackedPoint::observations_, localmap.h:276) is filled by Frame::Commit in
// frame order (localmap.cpp:85-89), so here it is the point's observations in ascending frame index,
// ties by map observation index.  The Eigen pieces (Quaterniond::matrix, inverse, _transformVector,
// quaternion-from-matrix, 3x3 inverse) are written out as Eigen 3.2 computes them.
#include <cmath>
#include <cstdint>
#include <vector>
#include <algorithm>

#include "slamgpu.h"

namespace {

constexpr int kBadLocation = 1 << SG_BAD_LOCATION;
constexpr int kNoBaseline = 1 << SG_NO_BASELINE;
constexpr int kNoObservations = 1 << SG_NO_OBSERVATIONS;
constexpr int kMismatched = 1 << SG_MISMATCHED;
constexpr int kBadFeature = 1 << SG_BAD_FEATURE;

bool SlamUsable(int f) {   // localmap.h:240-246
  return !(f & kBadLocation) && !(f & kNoBaseline) && !(f & kNoObservations) && !(f & kBadFeature);
}
bool FeatureUsable(int f) { return !(f & kMismatched) && !(f & kBadLocation); }   // localmap.h:247

// Per point: its observations in TrackedPoint::observations() order.
std::vector<std::vector<int>> PointObs(const sg_map* m) {
  std::vector<std::vector<int>> po(m->num_points);
  std::vector<int> order(m->num_obs);
  for (int o = 0; o < m->num_obs; ++o) order[o] = o;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return m->obs_frame[a] < m->obs_frame[b]; });
  for (int o : order) po[m->obs_point[o]].push_back(o);
  return po;
}

// Eigen QuaternionBase::_transformVector: v + w (2 q.vec x v) + q.vec x (2 q.vec x v).
void QuatRotate(const double* q, const double* v, double* out) {
  double uv0 = q[1] * v[2] - q[2] * v[1], uv1 = q[2] * v[0] - q[0] * v[2], uv2 = q[0] * v[1] - q[1] * v[0];
  uv0 += uv0; uv1 += uv1; uv2 += uv2;
  out[0] = v[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
  out[1] = v[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
  out[2] = v[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
}

// Eigen QuaternionBase::toRotationMatrix.
void QuatMatrix(const double* q, double R[3][3]) {
  const double x = q[0], y = q[1], z = q[2], w = q[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz;       R[0][2] = txz + twy;
  R[1][0] = txy + twz;       R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
  R[2][0] = txz - twy;       R[2][1] = tyz + twx;       R[2][2] = 1 - (txx + tyy);
}

// Eigen QuaternionBase::inverse (conjugate / squared norm).
void QuatInverse(const double* q, double* out) {
  const double n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  if (n2 > 0) {
    out[0] = -q[0] / n2; out[1] = -q[1] / n2; out[2] = -q[2] / n2; out[3] = q[3] / n2;
  } else {
    out[0] = out[1] = out[2] = out[3] = 0;
  }
}

// Camera::PixelToPlane (localmap.h:52-73).
void PixelToPlane(const double* k, const double* p, double* out) {
  double xp = p[0], yp = p[1];
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

// TrackedPoint::CheckFlags (localmap.cpp:44-83).
void CheckFlags(const sg_map* m, const std::vector<int>& obs, int* flags) {
  if (*flags & kNoObservations) {
    int good = 0;
    for (int o : obs) {
      if (m->obs_disabled[o]) continue;
      if (++good >= 2) {
        *flags &= ~kNoObservations;
        break;
      }
    }
  }
  if (*flags & kNoBaseline) {
    const double* base = nullptr;
    for (int o : obs) {
      if (m->obs_disabled[o]) continue;
      const double* pos = m->t + 3 * m->obs_frame[o];
      if (!base) {
        base = pos;
        continue;
      }
      const double d0 = pos[0] - base[0], d1 = pos[1] - base[1], d2 = pos[2] - base[2];
      if (std::sqrt(d0 * d0 + d1 * d1 + d2 * d2) < 50) continue;
      *flags &= ~kNoBaseline;
      break;
    }
  }
}

}  // namespace

extern "C" {

// LocalMap::Clean(error_threshold) (localmap.cpp:283-398).  Reads obs_error (ReprojectMap); writes
// X[4p+3] (sign / magnitude fix), point_flags, point_uncertainty, obs_disabled.  Returns the reference's
// bool (false when observations were disabled).
int orm_clean(sg_map* m, double error_threshold) {
  const auto po = PointObs(m);
  int result = 1;
  std::vector<std::pair<double, int>> errmap;   // (err, observation): multimap<double, ...> content
  std::vector<char> changed(m->num_points, 0);
  for (int p = 0; p < m->num_points; ++p) {
    if (!SlamUsable(m->point_flags[p])) continue;
    double* loc = m->X + 4 * p;
    if (loc[3] < 0) loc[3] = -loc[3];
    if (std::fabs(loc[3]) < 1e-6) loc[3] = 1e-6;
    double sum_err = 0;
    for (int o : po[p]) {
      const double e0 = m->obs_error[2 * o], e1 = m->obs_error[2 * o + 1];
      const double err = std::sqrt(e0 * e0 + e1 * e1);
      sum_err += err;
      // pos = rotation * (position - translation), position = loc.head<3>() / loc[3]
      const int f = m->obs_frame[o];
      const double* t = m->t + 3 * f;
      const double v[3] = {loc[0] / loc[3] - t[0], loc[1] / loc[3] - t[1], loc[2] / loc[3] - t[2]};
      double pos[3];
      QuatRotate(m->q + 4 * f, v, pos);
      if (pos[2] < 1) {
        m->point_flags[p] |= kBadLocation;
        changed[p] = 1;
        break;
      }
      if (!m->obs_disabled[o] && err > error_threshold) errmap.push_back({err, o});
    }
    const int nobs = (int)po[p].size();
    const double avg_err = sum_err / nobs;
    if (avg_err > 1.5 && nobs > 4) {
      m->point_flags[p] |= kBadFeature;
      changed[p] = 1;
    }
    m->point_uncertainty[p] = avg_err;
  }
  if (!errmap.empty()) {
    double maxerr = 0;
    for (const auto& e : errmap) maxerr = std::max(maxerr, e.first);
    maxerr = std::max(error_threshold, maxerr / 4.);
    for (const auto& e : errmap) {   // every entry not below maxerr is reached by the worst-first walk
      if (e.first < maxerr) continue;
      const int o = e.second;
      if (m->obs_disabled[o]) continue;
      m->obs_disabled[o] = 1;
      const int p = m->obs_point[o];
      m->point_flags[p] |= kMismatched;
      changed[p] = 1;
      result = 0;
    }
  }
  for (int p = 0; p < m->num_points; ++p) {
    if (!changed[p]) continue;
    m->point_flags[p] |= kNoObservations | kNoBaseline;
    CheckFlags(m, po[p], &m->point_flags[p]);
  }
  return result;
}

// LocalMap::ApplyEpipolarConstraint (localmap.cpp:232-276) with EssentialMatrix (211-230).  Writes
// point_flags and obs_disabled.  Returns the number of points whose |r| exceeded the 0.15 cut.
int orm_apply_epipolar(sg_map* m) {
  const auto po = PointObs(m);
  int hits = 0;
  for (int p = 0; p < m->num_points; ++p) {
    const auto& obs = po[p];
    const int n = (int)obs.size();
    if (n < 2) continue;
    const int fl = m->point_flags[p];
    if (!FeatureUsable(fl)) continue;
    if (fl & kBadFeature) continue;
    const int o1 = obs[n - 1];
    int o2 = obs[n - 2];
    for (int i = 3; i < n && m->obs_disabled[o2]; ++i) o2 = obs[n - i];
    const int f1 = m->obs_frame[o1], f2 = m->obs_frame[o2];
    if (m->frame_camera[f1] == m->frame_camera[f2] || m->obs_disabled[o2]) continue;
    double p1[2], p2[2];
    PixelToPlane(m->k + 7 * m->frame_camera[f1], m->obs_pt + 2 * o1, p1);
    PixelToPlane(m->k + 7 * m->frame_camera[f2], m->obs_pt + 2 * o2, p2);
    const double h1[3] = {p1[0], p1[1], 1}, h2[3] = {p2[0], p2[1], 1};
    // EssentialMatrix(from = obs1 frame, to = obs2 frame): E = (R_to R_from^-1) [t_to - t_from]_x (normalised t)
    double Rt[3][3], Rf[3][3], qi[4];
    QuatMatrix(m->q + 4 * f2, Rt);
    QuatInverse(m->q + 4 * f1, qi);
    QuatMatrix(qi, Rf);
    double rot[3][3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) rot[i][j] = Rt[i][0] * Rf[0][j] + Rt[i][1] * Rf[1][j] + Rt[i][2] * Rf[2][j];
    double tr[3] = {m->t[3 * f2] - m->t[3 * f1], m->t[3 * f2 + 1] - m->t[3 * f1 + 1], m->t[3 * f2 + 2] - m->t[3 * f1 + 2]};
    const double tn = std::sqrt(tr[0] * tr[0] + tr[1] * tr[1] + tr[2] * tr[2]);
    if (tn > 0) { tr[0] /= tn; tr[1] /= tn; tr[2] /= tn; }
    const double sk[3][3] = {{0, -tr[2], tr[1]}, {tr[2], 0, -tr[0]}, {-tr[1], tr[0], 0}};
    double E[3][3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) E[i][j] = rot[i][0] * sk[0][j] + rot[i][1] * sk[1][j] + rot[i][2] * sk[2][j];
    double r = 0;
    for (int i = 0; i < 3; ++i) r += h2[i] * (E[i][0] * h1[0] + E[i][1] * h1[1] + E[i][2] * h1[2]);
    const double threshold = 0.0015;
    if (std::fabs(r) > threshold * 100) {
      ++hits;
      if (n > 8) {
        m->obs_disabled[o1] = 1;
        m->point_flags[p] |= kMismatched;
      } else {
        m->point_flags[p] |= kBadFeature;
      }
    }
  }
  return hits;
}

// LocalMap::Normalize (localmap.cpp:114-155).  xlate = -t0, scale = 1 (line 125 overrides the 150 mm
// baseline scale); every frame's translation and every point are moved by xlate (TrackedPoint::move
// adds xlate * w, rescale(1 / scale) normalises the 4-vector); then rotate = q0.matrix(), each frame's rotation
// becomes quaternion(R_f * rotate^-1) (Quaternion * Matrix3 is a matrix product, assigned back through
// quaternionbase_assign_impl), each translation and point direction is multiplied by rotate.
void orm_normalize(sg_map* m) {
  if (m->num_frames < 2) return;
  const double xl[3] = {-m->t[0], -m->t[1], -m->t[2]};
  for (int f = 0; f < m->num_frames; ++f)
    for (int c = 0; c < 3; ++c) m->t[3 * f + c] += xl[c];
  for (int p = 0; p < m->num_points; ++p) {
    double* x = m->X + 4 * p;
    for (int c = 0; c < 3; ++c) x[c] += xl[c] * x[3];
    const double nrm = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
    for (int c = 0; c < 4; ++c) x[c] /= nrm;
  }
  double R[3][3], inv[3][3];
  QuatMatrix(m->q, R);
  {
    // compute_inverse_size3_helper: cofactors, determinant along column 0
    auto cof = [&](int i, int j) {
      const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      return R[i1][j1] * R[i2][j2] - R[i1][j2] * R[i2][j1];
    };
    const double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    const double invdet = 1.0 / (c0 * R[0][0] + c1 * R[1][0] + c2 * R[2][0]);
    inv[0][0] = c0 * invdet; inv[0][1] = c1 * invdet; inv[0][2] = c2 * invdet;
    inv[1][0] = cof(0, 1) * invdet; inv[1][1] = cof(1, 1) * invdet; inv[1][2] = cof(2, 1) * invdet;
    inv[2][0] = cof(0, 2) * invdet; inv[2][1] = cof(1, 2) * invdet; inv[2][2] = cof(2, 2) * invdet;
  }
  for (int f = 0; f < m->num_frames; ++f) {
    double Rf[3][3], M[3][3];
    QuatMatrix(m->q + 4 * f, Rf);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) M[i][j] = Rf[i][0] * inv[0][j] + Rf[i][1] * inv[1][j] + Rf[i][2] * inv[2][j];
    double* q = m->q + 4 * f;
    // quaternionbase_assign_impl<Matrix3>: trace branch, else the largest diagonal
    double t = M[0][0] + M[1][1] + M[2][2];
    if (t > 0.0) {
      t = std::sqrt(t + 1.0);
      q[3] = 0.5 * t;
      t = 0.5 / t;
      q[0] = (M[2][1] - M[1][2]) * t;
      q[1] = (M[0][2] - M[2][0]) * t;
      q[2] = (M[1][0] - M[0][1]) * t;
    } else {
      int i = 0;
      if (M[1][1] > M[0][0]) i = 1;
      if (M[2][2] > M[i][i]) i = 2;
      const int j = (i + 1) % 3, k = (j + 1) % 3;
      t = std::sqrt(M[i][i] - M[j][j] - M[k][k] + 1.0);
      q[i] = 0.5 * t;
      t = 0.5 / t;
      q[3] = (M[k][j] - M[j][k]) * t;
      q[j] = (M[j][i] + M[i][j]) * t;
      q[k] = (M[k][i] + M[i][k]) * t;
    }
    double* tf = m->t + 3 * f;
    const double v[3] = {tf[0], tf[1], tf[2]};
    for (int i = 0; i < 3; ++i) tf[i] = R[i][0] * v[0] + R[i][1] * v[1] + R[i][2] * v[2];
  }
  for (int p = 0; p < m->num_points; ++p) {
    double* x = m->X + 4 * p;
    const double v[3] = {x[0], x[1], x[2]};
    for (int i = 0; i < 3; ++i) x[i] = R[i][0] * v[0] + R[i][1] * v[1] + R[i][2] * v[2];
  }
}

}  // extern "C"
