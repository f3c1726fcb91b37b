// map_ops.hip — LocalMap maintenance on the device, run on the BA residuals after every solve
// (main.cpp:584-605):
//   LocalMap::Clean(error_threshold)      localmap.cpp:283-398 (+ TrackedPoint::CheckFlags 44-83)
//   LocalMap::ApplyEpipolarConstraint()   localmap.cpp:232-276 (+ EssentialMatrix 211-230)
//   LocalMap::Normalize()                 localmap.cpp:114-155 (gauge: frame 0 to the origin and to the
//                                         identity rotation; main.cpp:602-605 runs it between two ReprojectMap)
//
// Both are independent per point once a point's observations are listed in TrackedPoint::observations()
// order (ascending frame index: Frame::Commit adds them frame by frame, localmap.cpp:85-89).  The only
// global step is Clean's worst-error cut max(threshold, max err / 4) over the candidates of all points:
// a per-workgroup maximum, then one atomicMax on the bit pattern (non-negative doubles order as their
// bits), so the result is independent of scheduling.  One thread per point; the map's own arrays are
// uploaded per call (the caller owns the LocalMap) and the mutated ones copied back.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "map_ops.h"

namespace sg {

namespace {

constexpr int kThreads = 256;
constexpr int kBadLocation = 1 << SG_BAD_LOCATION;
constexpr int kNoBaseline = 1 << SG_NO_BASELINE;
constexpr int kNoObservations = 1 << SG_NO_OBSERVATIONS;
constexpr int kMismatched = 1 << SG_MISMATCHED;
constexpr int kBadFeature = 1 << SG_BAD_FEATURE;

struct MapDev {
  const double* k;
  const double* q;
  const double* t;
  const int32_t* frame_cam;
  double* X;
  int32_t* flags;
  double* unc;
  const double* obs_pt;
  const double* obs_err;
  const int32_t* obs_frame;
  int32_t* obs_dis;
  const int32_t* poff;   // [P+1] per point, its observations in TrackedPoint::observations() order
  const int32_t* pobs;   // [M]
  uint8_t* cand;         // [M] Clean: observation entered the worst-error list
  uint8_t* changed;      // [P] Clean: point goes through CheckFlags
  unsigned long long* maxbits;   // Clean: bit pattern of the largest candidate error
  int32_t* counters;     // [0] Clean result (1 = nothing disabled), [1] epipolar hits
  int P;
};

__device__ __forceinline__ bool slam_usable(int f) {   // localmap.h:240-246
  return !(f & kBadLocation) && !(f & kNoBaseline) && !(f & kNoObservations) && !(f & kBadFeature);
}

// Eigen QuaternionBase::_transformVector.
__device__ __forceinline__ void quat_rotate(const double* q, const double* v, double* out) {
  double uv0 = q[1] * v[2] - q[2] * v[1], uv1 = q[2] * v[0] - q[0] * v[2], uv2 = q[0] * v[1] - q[1] * v[0];
  uv0 += uv0;
  uv1 += uv1;
  uv2 += uv2;
  out[0] = v[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
  out[1] = v[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
  out[2] = v[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
}

// Eigen QuaternionBase::toRotationMatrix.
__device__ __forceinline__ void quat_matrix(const double* q, double R[3][3]) {
  const double x = q[0], y = q[1], z = q[2], w = q[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz;       R[0][2] = txz + twy;
  R[1][0] = txy + twz;       R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
  R[2][0] = txz - twy;       R[2][1] = tyz + twx;       R[2][2] = 1 - (txx + tyy);
}

// Camera::PixelToPlane (localmap.h:52-73): three fixed-point undistortion steps.
__device__ __forceinline__ void pixel_to_plane(const double* k, double px, double py, double* out) {
  double xp = (px - k[5]) / k[3], yp = (py - k[6]) / k[4];
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

__device__ __forceinline__ double obs_err_norm(const MapDev& d, int o) {
  const double e0 = d.obs_err[2 * o], e1 = d.obs_err[2 * o + 1];
  return sqrt(e0 * e0 + e1 * e1);
}

// Clean, per point: location fix, error walk (BAD_LOCATION break), worst-error candidates, BAD_FEATURE,
// uncertainty; then the workgroup / global maximum of the candidate errors.
__global__ __launch_bounds__(kThreads) void k_clean_walk(MapDev d, double thr) {
  __shared__ double red[kThreads / 64];
  const int p = blockIdx.x * kThreads + threadIdx.x;
  double mx = 0.0;
  if (p < d.P && slam_usable(d.flags[p])) {
    int fl = d.flags[p];
    double* loc = d.X + 4 * (size_t)p;
    double w = loc[3];
    if (w < 0) w = -w;
    if (fabs(w) < 1e-6) w = 1e-6;
    loc[3] = w;
    const double px = loc[0] / w, py = loc[1] / w, pz = loc[2] / w;
    const int o0 = d.poff[p], o1 = d.poff[p + 1];
    bool ch = false;
    double sum_err = 0;
    for (int i = o0; i < o1; ++i) {
      const int o = d.pobs[i];
      const double err = obs_err_norm(d, o);
      sum_err += err;
      const int f = d.obs_frame[o];
      const double* t = d.t + 3 * f;
      const double v[3] = {px - t[0], py - t[1], pz - t[2]};
      double pos[3];
      quat_rotate(d.q + 4 * f, v, pos);
      if (pos[2] < 1) {
        fl |= kBadLocation;
        ch = true;
        break;
      }
      if (!d.obs_dis[o] && err > thr) {
        d.cand[o] = 1;
        mx = fmax(mx, err);
      }
    }
    const int nobs = o1 - o0;
    const double avg_err = sum_err / nobs;
    if (avg_err > 1.5 && nobs > 4) {
      fl |= kBadFeature;
      ch = true;
    }
    d.unc[p] = avg_err;
    d.flags[p] = fl;
    d.changed[p] = ch ? 1 : 0;
  }
  // workgroup max, then one atomic per workgroup (errors are >= 0: their bit patterns order like them)
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) mx = fmax(mx, __shfl_xor(mx, m));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    double b = red[0];
    for (int i = 1; i < kThreads / 64; ++i) b = fmax(b, red[i]);
    if (b > 0.0) atomicMax(d.maxbits, (unsigned long long)__double_as_longlong(b));
  }
}

// TrackedPoint::CheckFlags (localmap.cpp:44-83).
__device__ __forceinline__ int check_flags(const MapDev& d, int o0, int o1, int fl) {
  if (fl & kNoObservations) {
    int good = 0;
    for (int i = o0; i < o1; ++i) {
      if (d.obs_dis[d.pobs[i]]) continue;
      if (++good >= 2) {
        fl &= ~kNoObservations;
        break;
      }
    }
  }
  if (fl & kNoBaseline) {
    int base = -1;
    for (int i = o0; i < o1; ++i) {
      const int o = d.pobs[i];
      if (d.obs_dis[o]) continue;
      const int f = d.obs_frame[o];
      if (base < 0) {
        base = f;
        continue;
      }
      const double d0 = d.t[3 * f] - d.t[3 * base], d1 = d.t[3 * f + 1] - d.t[3 * base + 1],
                   d2 = d.t[3 * f + 2] - d.t[3 * base + 2];
      if (sqrt(d0 * d0 + d1 * d1 + d2 * d2) < 50) continue;
      fl &= ~kNoBaseline;
      break;
    }
  }
  return fl;
}

// Clean, per point: disable the candidates at or above the cut (the worst-first walk of the reference
// reaches exactly those), MISMATCHED, then NO_OBSERVATIONS | NO_BASELINE + CheckFlags on changed points.
__global__ __launch_bounds__(kThreads) void k_clean_cut(MapDev d, double thr) {
  const int p = blockIdx.x * kThreads + threadIdx.x;
  if (p >= d.P) return;
  const unsigned long long mb = *d.maxbits;
  const double cut = fmax(thr, __longlong_as_double((long long)mb) / 4.);
  int fl = d.flags[p];
  bool ch = d.changed[p] != 0;
  const int o0 = d.poff[p], o1 = d.poff[p + 1];
  if (mb != 0ull) {
    for (int i = o0; i < o1; ++i) {
      const int o = d.pobs[i];
      if (!d.cand[o]) continue;
      if (obs_err_norm(d, o) < cut) continue;
      if (d.obs_dis[o]) continue;
      d.obs_dis[o] = 1;
      fl |= kMismatched;
      ch = true;
      d.counters[0] = 0;
    }
  }
  if (ch) fl = check_flags(d, o0, o1, fl | kNoObservations | kNoBaseline);
  d.flags[p] = fl;
}

// ApplyEpipolarConstraint, per point: the last observation against the latest enabled earlier one of the
// other camera (the reference's search stops before the point's first observation), r = h2^T E h1 with
// E = (R_to R_from^-1) [t_to - t_from]_x, |r| > 0.15 disables the last observation (> 8 observations,
// MISMATCHED) or marks BAD_FEATURE.
__global__ __launch_bounds__(kThreads) void k_epipolar(MapDev d) {
  const int p = blockIdx.x * kThreads + threadIdx.x;
  if (p >= d.P) return;
  const int o0 = d.poff[p], n = d.poff[p + 1] - o0;
  if (n < 2) return;
  const int fl = d.flags[p];
  if ((fl & kMismatched) || (fl & kBadLocation)) return;   // !feature_usable()
  if (fl & kBadFeature) return;
  const int o1 = d.pobs[o0 + n - 1];
  int o2 = d.pobs[o0 + n - 2];
  for (int i = 3; i < n && d.obs_dis[o2]; ++i) o2 = d.pobs[o0 + n - i];
  const int f1 = d.obs_frame[o1], f2 = d.obs_frame[o2];
  if (d.frame_cam[f1] == d.frame_cam[f2] || d.obs_dis[o2]) return;
  double p1[2], p2[2];
  pixel_to_plane(d.k + 7 * d.frame_cam[f1], d.obs_pt[2 * o1], d.obs_pt[2 * o1 + 1], p1);
  pixel_to_plane(d.k + 7 * d.frame_cam[f2], d.obs_pt[2 * o2], d.obs_pt[2 * o2 + 1], p2);
  const double h1[3] = {p1[0], p1[1], 1}, h2[3] = {p2[0], p2[1], 1};
  const double* qf = d.q + 4 * f1;
  const double n2 = qf[0] * qf[0] + qf[1] * qf[1] + qf[2] * qf[2] + qf[3] * qf[3];
  double qi[4] = {0, 0, 0, 0};
  if (n2 > 0) {
    qi[0] = -qf[0] / n2;
    qi[1] = -qf[1] / n2;
    qi[2] = -qf[2] / n2;
    qi[3] = qf[3] / n2;
  }
  double Rt[3][3], Rf[3][3], rot[3][3];
  quat_matrix(d.q + 4 * f2, Rt);
  quat_matrix(qi, Rf);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) rot[i][j] = Rt[i][0] * Rf[0][j] + Rt[i][1] * Rf[1][j] + Rt[i][2] * Rf[2][j];
  double tr[3] = {d.t[3 * f2] - d.t[3 * f1], d.t[3 * f2 + 1] - d.t[3 * f1 + 1], d.t[3 * f2 + 2] - d.t[3 * f1 + 2]};
  const double tn = sqrt(tr[0] * tr[0] + tr[1] * tr[1] + tr[2] * tr[2]);
  if (tn > 0) {
    tr[0] /= tn;
    tr[1] /= tn;
    tr[2] /= tn;
  }
  const double sk[3][3] = {{0, -tr[2], tr[1]}, {tr[2], 0, -tr[0]}, {-tr[1], tr[0], 0}};
  double r = 0;
  for (int i = 0; i < 3; ++i) {
    double e[3];
    for (int j = 0; j < 3; ++j) e[j] = rot[i][0] * sk[0][j] + rot[i][1] * sk[1][j] + rot[i][2] * sk[2][j];
    r += h2[i] * (e[0] * h1[0] + e[1] * h1[1] + e[2] * h1[2]);
  }
  if (fabs(r) > 0.0015 * 100) {
    atomicAdd(d.counters + 1, 1);
    if (n > 8) {
      d.obs_dis[o1] = 1;
      d.flags[p] = fl | kMismatched;
    } else {
      d.flags[p] = fl | kBadFeature;
    }
  }
}

// ---- LocalMap::Normalize (localmap.cpp:114-155) with Eigen 3.2's arithmetic written out.

// quaternionbase_assign_impl<Matrix3>: the trace branch, else the largest-diagonal branch.
__device__ __forceinline__ void quat_from_matrix(const double m[3][3], double* q) {
  double t = m[0][0] + m[1][1] + m[2][2];
  if (t > 0.0) {
    t = sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (m[2][1] - m[1][2]) * t;
    q[1] = (m[0][2] - m[2][0]) * t;
    q[2] = (m[1][0] - m[0][1]) * t;
  } else {
    int i = 0;
    if (m[1][1] > m[0][0]) i = 1;
    if (m[2][2] > m[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m[k][j] - m[j][k]) * t;
    q[j] = (m[j][i] + m[i][j]) * t;
    q[k] = (m[k][i] + m[i][k]) * t;
  }
}

// compute_inverse_size3_helper: cofactors, determinant along column 0.
__device__ __forceinline__ void inverse3(const double m[3][3], double r[3][3]) {
  auto cof = [&](int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1];
  };
  const double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
  const double invdet = 1.0 / (c0 * m[0][0] + c1 * m[1][0] + c2 * m[2][0]);
  r[0][0] = c0 * invdet;
  r[0][1] = c1 * invdet;
  r[0][2] = c2 * invdet;
  r[1][0] = cof(0, 1) * invdet;
  r[1][1] = cof(1, 1) * invdet;
  r[1][2] = cof(2, 1) * invdet;
  r[2][0] = cof(0, 2) * invdet;
  r[2][1] = cof(1, 2) * invdet;
  r[2][2] = cof(2, 2) * invdet;
}

struct NormArgs {
  double q0[4], t0[3];   // frame 0's pose before the call (every thread reads it, frame 0's thread rewrites it)
};

// Threads [0, F): frames; threads [F, F + P): points.  scale = 1 in the reference (localmap.cpp:125), so its
// multiplications by scale are identities and are not performed.
__global__ __launch_bounds__(kThreads) void k_normalize(NormArgs a, double* q, double* t, double* X, int F, int P) {
  const int id = blockIdx.x * kThreads + threadIdx.x;
  if (id >= F + P) return;
  const double xl[3] = {-a.t0[0], -a.t0[1], -a.t0[2]};
  double R[3][3];
  quat_matrix(a.q0, R);   // rotate = pose1->rotation().matrix()
  if (id < F) {
    double* tf = t + 3 * id;
    double v[3] = {tf[0] + xl[0], tf[1] + xl[1], tf[2] + xl[2]};
    double inv[3][3], Rf[3][3], M[3][3];
    inverse3(R, inv);
    quat_matrix(q + 4 * id, Rf);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) M[i][j] = Rf[i][0] * inv[0][j] + Rf[i][1] * inv[1][j] + Rf[i][2] * inv[2][j];
    double qn[4];
    quat_from_matrix(M, qn);
    for (int c = 0; c < 4; ++c) q[4 * id + c] = qn[c];
    for (int i = 0; i < 3; ++i) tf[i] = R[i][0] * v[0] + R[i][1] * v[1] + R[i][2] * v[2];
  } else {
    double* x = X + 4 * (size_t)(id - F);
    double v[4] = {x[0] + xl[0] * x[3], x[1] + xl[1] * x[3], x[2] + xl[2] * x[3], x[3]};   // move(xlate)
    const double nrm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);    // normalize()
    for (int c = 0; c < 4; ++c) v[c] /= nrm;
    for (int i = 0; i < 3; ++i) x[i] = R[i][0] * v[0] + R[i][1] * v[1] + R[i][2] * v[2];
    x[3] = v[3];
  }
}

}  // namespace

MapOps::MapOps(const sg_device_options& dev, hipStream_t stream) : dev_(dev) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) throw Error(SG_ENODEV, "no HIP device available");
  SG_REQUIRE(dev.device >= 0 && dev.device < ndev, SG_ENODEV, "device ordinal out of range");
  SG_HIP_CHECK(hipSetDevice(dev.device));
  if (stream) {
    stream_ = stream;
  } else {
    SG_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    own_stream_ = true;
  }
}

MapOps::~MapOps() {
  if (own_stream_ && stream_) (void)hipStreamDestroy(stream_);
}

// Upload a LocalMap and list each point's observations in TrackedPoint::observations() order (two stable
// counting sorts: by frame, then by point).
void MapOps::Upload(const sg_map* m) {
  SG_REQUIRE(m, SG_EINVAL, "null map");
  SG_REQUIRE(m->num_cameras >= 0 && m->num_frames >= 0 && m->num_points >= 0 && m->num_obs >= 0, SG_EINVAL,
             "negative map sizes");
  const int F = m->num_frames, P = m->num_points, M = m->num_obs;
  for (int o = 0; o < M; ++o)
    SG_REQUIRE(m->obs_frame[o] >= 0 && m->obs_frame[o] < F && m->obs_point[o] >= 0 && m->obs_point[o] < P,
               SG_EINVAL, "observation frame / point index out of range");
  for (int f = 0; f < F; ++f)
    SG_REQUIRE(m->frame_camera[f] >= 0 && m->frame_camera[f] < m->num_cameras, SG_EINVAL,
               "frame camera index out of range");
  std::vector<int32_t> fcnt(F + 1, 0), byf(M);
  for (int o = 0; o < M; ++o) fcnt[m->obs_frame[o] + 1]++;
  for (int f = 0; f < F; ++f) fcnt[f + 1] += fcnt[f];
  for (int o = 0; o < M; ++o) byf[fcnt[m->obs_frame[o]]++] = o;
  std::vector<int32_t> poff(P + 1, 0), pobs(M);
  for (int o = 0; o < M; ++o) poff[m->obs_point[o] + 1]++;
  for (int p = 0; p < P; ++p) poff[p + 1] += poff[p];
  {
    std::vector<int32_t> fill(poff.begin(), poff.end() - 1);
    for (int i = 0; i < M; ++i) pobs[fill[m->obs_point[byf[i]]]++] = byf[i];
  }
  hipStream_t s = stream_;
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  io_.Begin();
  io_.Up(k_, m->k, 7 * (size_t)m->num_cameras);
  io_.Up(q_, m->q, 4 * (size_t)F);
  io_.Up(t_, m->t, 3 * (size_t)F);
  io_.Up(fcam_, m->frame_camera, (size_t)F);
  io_.Up(X_, m->X, 4 * (size_t)P);
  io_.Up(flags_, m->point_flags, (size_t)P);
  io_.Up(unc_, m->point_uncertainty, (size_t)P);
  io_.Up(obs_pt_, m->obs_pt, 2 * (size_t)M);
  io_.Up(obs_err_, m->obs_error, 2 * (size_t)M);
  io_.Up(obs_frame_, m->obs_frame, (size_t)M);
  io_.Up(obs_dis_, m->obs_disabled, (size_t)M);
  io_.Up(poff_, poff);
  io_.Up(pobs_, pobs);
  io_.UpZero(cand_, (size_t)M);
  io_.UpZero(changed_, (size_t)P);
  io_.UpZero(scal_, 2);
  io_.Up(counters_, std::vector<int32_t>{1, 0});
  io_.FlushUp(s);
  P_ = P;
  M_ = M;
}

void MapOps::Download(sg_map* m, bool X, bool unc) {
  if (X) io_.Down(m->X, X_.ptr, 32 * (size_t)P_);
  if (unc) io_.Down(m->point_uncertainty, unc_.ptr, 8 * (size_t)P_);
  io_.Down(m->point_flags, flags_.ptr, 4 * (size_t)P_);
  io_.Down(m->obs_disabled, obs_dis_.ptr, 4 * (size_t)M_);
  io_.Down(counters_h_, counters_.ptr, 8);
  io_.FinishDown(stream_);
}

static MapDev MakeMapDev(DBuf<double>& k, DBuf<double>& q, DBuf<double>& t, DBuf<int32_t>& fcam, DBuf<double>& X,
                         DBuf<int32_t>& flags, DBuf<double>& unc, DBuf<double>& obs_pt, DBuf<double>& obs_err,
                         DBuf<int32_t>& obs_frame, DBuf<int32_t>& obs_dis, DBuf<int32_t>& poff,
                         DBuf<int32_t>& pobs, DBuf<uint8_t>& cand, DBuf<uint8_t>& changed,
                         DBuf<unsigned long long>& scal, DBuf<int32_t>& counters, int P) {
  MapDev d{};
  d.k = k.ptr;
  d.q = q.ptr;
  d.t = t.ptr;
  d.frame_cam = fcam.ptr;
  d.X = X.ptr;
  d.flags = flags.ptr;
  d.unc = unc.ptr;
  d.obs_pt = obs_pt.ptr;
  d.obs_err = obs_err.ptr;
  d.obs_frame = obs_frame.ptr;
  d.obs_dis = obs_dis.ptr;
  d.poff = poff.ptr;
  d.pobs = pobs.ptr;
  d.cand = cand.ptr;
  d.changed = changed.ptr;
  d.maxbits = scal.ptr;
  d.counters = counters.ptr;
  d.P = P;
  return d;
}

int MapOps::Clean(sg_map* m, double error_threshold) {
  Upload(m);
  const MapDev d = MakeMapDev(k_, q_, t_, fcam_, X_, flags_, unc_, obs_pt_, obs_err_, obs_frame_, obs_dis_, poff_,
                              pobs_, cand_, changed_, scal_, counters_, P_);
  if (P_ > 0) {
    const int nb = (P_ + kThreads - 1) / kThreads;
    hipLaunchKernelGGL(k_clean_walk, dim3(nb), dim3(kThreads), 0, stream_, d, error_threshold);
    hipLaunchKernelGGL(k_clean_cut, dim3(nb), dim3(kThreads), 0, stream_, d, error_threshold);
    SG_HIP_CHECK(hipGetLastError());
  }
  Download(m, true, true);
  return counters_h_[0];
}

void MapOps::Normalize(sg_map* m) {
  SG_REQUIRE(m && m->num_frames >= 0 && m->num_points >= 0, SG_EINVAL, "bad map");
  if (m->num_frames < 2) return;   // localmap.cpp:115-116
  const int F = m->num_frames, P = m->num_points;
  hipStream_t s = stream_;
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  io_.Begin();
  io_.Up(q_, m->q, 4 * (size_t)F);
  io_.Up(t_, m->t, 3 * (size_t)F);
  io_.Up(X_, m->X, 4 * (size_t)P);
  io_.FlushUp(s);
  NormArgs a{};
  for (int c = 0; c < 4; ++c) a.q0[c] = m->q[c];
  for (int c = 0; c < 3; ++c) a.t0[c] = m->t[c];
  hipLaunchKernelGGL(k_normalize, dim3((F + P + kThreads - 1) / kThreads), dim3(kThreads), 0, s, a, q_.ptr, t_.ptr,
                     X_.ptr, F, P);
  SG_HIP_CHECK(hipGetLastError());
  io_.Down(m->q, q_.ptr, 32 * (size_t)F);
  io_.Down(m->t, t_.ptr, 24 * (size_t)F);
  io_.Down(m->X, X_.ptr, 32 * (size_t)P);
  io_.FinishDown(s);
}

int MapOps::ApplyEpipolarConstraint(sg_map* m) {
  Upload(m);
  const MapDev d = MakeMapDev(k_, q_, t_, fcam_, X_, flags_, unc_, obs_pt_, obs_err_, obs_frame_, obs_dis_, poff_,
                              pobs_, cand_, changed_, scal_, counters_, P_);
  if (P_ > 0) {
    hipLaunchKernelGGL(k_epipolar, dim3((P_ + kThreads - 1) / kThreads), dim3(kThreads), 0, stream_, d);
    SG_HIP_CHECK(hipGetLastError());
  }
  Download(m, false, false);
  return counters_h_[1];
}

}  // namespace sg
