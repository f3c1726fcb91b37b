// project_math.h — projection model and its analytic Jacobian (device code, also host-compilable for tests).
//
// Restates project.h:11-54 (ProjectPoint) on plain scalars, plus the exact partial derivatives that
// Ceres' AutoDiffCostFunction<ReprojectionError, 2, 4, 3, 7, 4> (slam.cpp:285-287) produces for it, and
// the ceres::QuaternionParameterization pieces (slam.cpp:312-313) applied to Eigen [x,y,z,w] memory.
// The reference evaluates these with 18-wide dual numbers; on MI355X the derivative is written out by
// hand (about 150 flops per observation instead of ~19x the value cost).
#ifndef SG_PROJECT_MATH_H_
#define SG_PROJECT_MATH_H_

#include <math.h>

#if defined(__HIPCC__)
#define SG_HD __host__ __device__ __forceinline__
#else
#define SG_HD inline
#endif

namespace sg {

// Point in camera frame (project.h:24): p = q * (X.xyz - t * X.w) with Eigen's _transformVector
// (uv = 2 q.vec x v; p = v + w uv + q.vec x uv).  Returns v too (needed by the Jacobian).
template <typename T>
SG_HD void CameraPoint(const T* q, const T* t, const T* X, T* v, T* p) {
  v[0] = X[0] - t[0] * X[3];
  v[1] = X[1] - t[1] * X[3];
  v[2] = X[2] - t[2] * X[3];
  T c0 = q[1] * v[2] - q[2] * v[1];
  T c1 = q[2] * v[0] - q[0] * v[2];
  T c2 = q[0] * v[1] - q[1] * v[0];
  c0 = c0 + c0; c1 = c1 + c1; c2 = c2 + c2;
  p[0] = (v[0] + q[3] * c0) + (q[1] * c2 - q[2] * c1);
  p[1] = (v[1] + q[3] * c1) + (q[2] * c0 - q[0] * c2);
  p[2] = (v[2] + q[3] * c2) + (q[0] * c1 - q[1] * c0);
}

// project.h:27-47.  Returns false on the behind-camera rejection p.z < 0.001 X.w.
template <typename T>
SG_HD bool Project(const T* q, const T* t, const T* k, const T* X, T* uv) {
  T v[3], p[3];
  CameraPoint(q, t, X, v, p);
  if (p[2] < T(0.001) * X[3]) return false;
  T xp = p[0] / p[2];
  T yp = p[1] / p[2];
  const T r2 = xp * xp + yp * yp;
  const T d = T(1) + r2 * (k[0] + r2 * (k[1] + r2 * k[2]));
  xp = xp * d; yp = yp * d;
  xp = xp * k[3]; yp = yp * k[4];
  uv[0] = xp + k[5];
  uv[1] = yp + k[6];
  return true;
}

// Value + analytic Jacobian of the projection.  Outputs (row-major, 2 rows):
//   Jq[2][4]  d(uv)/d(q memory [x,y,z,w])     (global, before the local parameterization; if Jq != nullptr)
//   Jt[2][3]  d(uv)/d(t)
//   Jk[2][7]  d(uv)/d(k)                        (only if Jk != nullptr)
//   JX[2][4]  d(uv)/d(X)
//   Jr[2][3]  d(uv)/d(delta): the rotation in ceres::QuaternionParameterization's tangent space at q, i.e.
//             Jq * QuatLocalJacobian(q), formed directly (if Jr != nullptr).  Ceres's Plus reads Eigen's
//             [x,y,z,w] memory as [w,x,y,z] (slam.cpp:312-313), so its tangent basis is permuted against
//             Eigen's rotation; worked out symbolically, dp/d(delta) = (R(q) + (|q|^2 - 1) I) A(v) with
//             A(v) = 2 [[v1, v2, 0], [-v0, 0, v2], [0, -v0, -v1]] (v = X.xyz - t X.w, R the matrix of Eigen's
//             _transformVector, exact for any |q|), so d(uv)/d(delta) = (G R + (|q|^2 - 1) G) A(v): 24 flops
//             instead of forming the 3x4 dp/dq (~50), G dp/dq (24 FMAs) and the 4x3 product (24 FMAs).
template <typename T>
SG_HD bool ProjectJacobian(const T* q, const T* t, const T* k, const T* X, T* uv, T* Jq, T* Jt, T* Jk,
                           T* JX, T* Jr = nullptr) {
  T v[3], p[3];
  CameraPoint(q, t, X, v, p);
  if (p[2] < T(0.001) * X[3]) return false;
  const T iz = T(1) / p[2];
  const T xn = p[0] * iz, yn = p[1] * iz;
  const T r2 = xn * xn + yn * yn;
  const T d = T(1) + r2 * (k[0] + r2 * (k[1] + r2 * k[2]));
  const T dd = k[0] + r2 * (T(2) * k[1] + T(3) * k[2] * r2);   // d(distort)/d(r2)
  // Forward value exactly as project.h (same rounding as Project()).
  {
    T xp = p[0] / p[2], yp = p[1] / p[2];
    const T rr = xp * xp + yp * yp;
    const T dist = T(1) + rr * (k[0] + rr * (k[1] + rr * k[2]));
    xp = xp * dist; yp = yp * dist;
    xp = xp * k[3]; yp = yp * k[4];
    uv[0] = xp + k[5];
    uv[1] = yp + k[6];
  }
  // d(uv)/d(xn,yn)
  const T a00 = k[3] * (d + T(2) * xn * xn * dd);
  const T a01 = k[3] * (T(2) * xn * yn * dd);
  const T a10 = k[4] * (T(2) * xn * yn * dd);
  const T a11 = k[4] * (d + T(2) * yn * yn * dd);
  // G = d(uv)/d(p) = A * [[iz, 0, -xn iz], [0, iz, -yn iz]]
  T G[2][3];
  G[0][0] = a00 * iz; G[0][1] = a01 * iz; G[0][2] = -(a00 * xn + a01 * yn) * iz;
  G[1][0] = a10 * iz; G[1][1] = a11 * iz; G[1][2] = -(a10 * xn + a11 * yn) * iz;
  // R = dp/dv = I + 2w[u]x + 2[u]x^2 ; u = q.xyz, w = q[3]
  const T ux = q[0], uy = q[1], uz = q[2], w = q[3];
  T R[3][3];
  R[0][0] = T(1) - T(2) * (uy * uy + uz * uz);
  R[0][1] = T(2) * (ux * uy - w * uz);
  R[0][2] = T(2) * (ux * uz + w * uy);
  R[1][0] = T(2) * (ux * uy + w * uz);
  R[1][1] = T(1) - T(2) * (ux * ux + uz * uz);
  R[1][2] = T(2) * (uy * uz - w * ux);
  R[2][0] = T(2) * (ux * uz - w * uy);
  R[2][1] = T(2) * (uy * uz + w * ux);
  R[2][2] = T(1) - T(2) * (ux * ux + uy * uy);
  // GR = G R
  T GR[2][3];
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 3; ++c) GR[r][c] = G[r][0] * R[0][c] + G[r][1] * R[1][c] + G[r][2] * R[2][c];
  const T Rt0 = GR[0][0] * t[0] + GR[0][1] * t[1] + GR[0][2] * t[2];
  const T Rt1 = GR[1][0] * t[0] + GR[1][1] * t[1] + GR[1][2] * t[2];
  if (Jq) {
    // dp/du = -2w[v]x + 2 (u v^T + (u.v) I - 2 v u^T) ;  dp/dw = 2 (u x v)
    const T udv = ux * v[0] + uy * v[1] + uz * v[2];
    const T uu[3] = {ux, uy, uz};
    T Pq[3][4];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Pq[i][j] = T(2) * (uu[i] * v[j] - T(2) * v[i] * uu[j] + (i == j ? udv : T(0)));
    // -2w [v]x : [v]x = [[0,-v2,v1],[v2,0,-v0],[-v1,v0,0]]
    Pq[0][1] += T(2) * w * v[2];
    Pq[0][2] -= T(2) * w * v[1];
    Pq[1][0] -= T(2) * w * v[2];
    Pq[1][2] += T(2) * w * v[0];
    Pq[2][0] += T(2) * w * v[1];
    Pq[2][1] -= T(2) * w * v[0];
    Pq[0][3] = T(2) * (uy * v[2] - uz * v[1]);
    Pq[1][3] = T(2) * (uz * v[0] - ux * v[2]);
    Pq[2][3] = T(2) * (ux * v[1] - uy * v[0]);
    for (int r = 0; r < 2; ++r)
      for (int c = 0; c < 4; ++c) Jq[4 * r + c] = G[r][0] * Pq[0][c] + G[r][1] * Pq[1][c] + G[r][2] * Pq[2][c];
  }
  if (Jr) {
    const T n1 = (ux * ux + uy * uy) + (uz * uz + w * w) - T(1);
    for (int r = 0; r < 2; ++r) {
      const T g0 = GR[r][0] + n1 * G[r][0], g1 = GR[r][1] + n1 * G[r][1], g2 = GR[r][2] + n1 * G[r][2];
      Jr[3 * r + 0] = T(2) * (g0 * v[1] - g1 * v[0]);
      Jr[3 * r + 1] = T(2) * (g0 * v[2] - g2 * v[0]);
      Jr[3 * r + 2] = T(2) * (g1 * v[2] - g2 * v[1]);
    }
  }
  for (int r = 0; r < 2; ++r) {
    for (int c = 0; c < 3; ++c) Jt[3 * r + c] = -X[3] * GR[r][c];
    for (int c = 0; c < 3; ++c) JX[4 * r + c] = GR[r][c];
  }
  JX[3] = -Rt0;
  JX[7] = -Rt1;
  if (Jk) {
    const T r4 = r2 * r2, r6 = r4 * r2;
    Jk[0] = k[3] * xn * r2; Jk[1] = k[3] * xn * r4; Jk[2] = k[3] * xn * r6;
    Jk[3] = d * xn; Jk[4] = T(0); Jk[5] = T(1); Jk[6] = T(0);
    Jk[7] = k[4] * yn * r2; Jk[8] = k[4] * yn * r4; Jk[9] = k[4] * yn * r6;
    Jk[10] = T(0); Jk[11] = d * yn; Jk[12] = T(0); Jk[13] = T(1);
  }
  return true;
}

// ceres::QuaternionParameterization::ComputeJacobian on Eigen memory x (row-major 4x3).
template <typename T>
SG_HD void QuatLocalJacobian(const T* x, T* L) {
  L[0] = -x[1]; L[1] = -x[2]; L[2] = -x[3];
  L[3] = x[0];  L[4] = x[3];  L[5] = -x[2];
  L[6] = -x[3]; L[7] = x[0];  L[8] = x[1];
  L[9] = x[2];  L[10] = -x[1]; L[11] = x[0];
}

// ceres::QuaternionParameterization::Plus on Eigen memory x.
template <typename T>
SG_HD void QuatPlus(const T* x, const T* d, T* out) {
  const T nd = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd > T(0)) {
    const T s = sin(nd) / nd;
    const T z0 = cos(nd), z1 = s * d[0], z2 = s * d[1], z3 = s * d[2];
    out[0] = z0 * x[0] - z1 * x[1] - z2 * x[2] - z3 * x[3];
    out[1] = z0 * x[1] + z1 * x[0] + z2 * x[3] - z3 * x[2];
    out[2] = z0 * x[2] - z1 * x[3] + z2 * x[0] + z3 * x[1];
    out[3] = z0 * x[3] + z1 * x[2] - z2 * x[1] + z3 * x[0];
  } else {
    out[0] = x[0]; out[1] = x[1]; out[2] = x[2]; out[3] = x[3];
  }
}

// ceres::CauchyLoss(a) (b = a^2): rho0 = b log(1 + s/b), rho1 = 1/(1 + s/b).
template <typename T>
SG_HD void Cauchy(T s, T b, T inv_b, T* rho0, T* rho1) {
  const T sum = T(1) + s * inv_b;
  *rho1 = T(1) / sum;
  *rho0 = b * log(sum);
}

// Local (corrected) Jacobian of one ReprojectionError block: returns the corrected residual r~ (2),
// camera part Jc[2][6] = [d/drot_local(3), d/dt(3)], point part Jp[2][4], and cost 0.5 rho.
template <typename T>
SG_HD bool LinearizeObservation(const T* q, const T* t, const T* k, const T* X, const T* pt, T b, T inv_b,
                                T* r, T* Jc, T* Jp, T* cost, T* Jk = nullptr) {
  T uv[2], Jr[6], Jt[6], JX[8];
  if (!ProjectJacobian(q, t, k, X, uv, (T*)nullptr, Jt, Jk, JX, Jr)) return false;
  const T r0 = uv[0] - pt[0], r1 = uv[1] - pt[1];
  T rho0, rho1;
  Cauchy(r0 * r0 + r1 * r1, b, inv_b, &rho0, &rho1);
  *cost = T(0.5) * rho0;
  const T sr = sqrt(rho1);
  r[0] = sr * r0;
  r[1] = sr * r1;
  // d(uv)/dt = -X.w d(uv)/d(X.xyz) (ProjectJacobian: Jt = -X.w GR, JX[:, 0:3] = GR), so the corrected translation
  // columns are formed from the corrected point columns, -X.w J~p[:, c]: the device stores J~p only and every reader
  // recomputes the translation columns with this same product (ba_device.h jc_from_pairs), bit for bit
  (void)Jt;
  for (int i = 0; i < 2; ++i) {
    for (int c = 0; c < 3; ++c) Jc[6 * i + c] = sr * Jr[3 * i + c];
    for (int c = 0; c < 4; ++c) Jp[4 * i + c] = sr * JX[4 * i + c];
    for (int c = 0; c < 3; ++c) Jc[6 * i + 3 + c] = -X[3] * Jp[4 * i + c];
  }
  if (Jk)
    for (int c = 0; c < 14; ++c) Jk[c] *= sr;
  return true;
}

}  // namespace sg

#endif  // SG_PROJECT_MATH_H_
