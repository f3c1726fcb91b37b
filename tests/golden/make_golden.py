"""Generate the committed golden fixtures for the bundle-adjustment path (run from the repo root).

The reference (ywrt/slam-robot) holds no fixtures for this path and cannot be built here, so the pins are:
  1. c1_ba.npz — the oracle's (CPU restatement, oracle/oracle_ba.cpp) solve of the C1 scene, seed 1: a
     regression pin for the oracle and the parity target for the device solver; plus a scipy check that the
     oracle's converged state is a local minimum (scipy started there does not descend further), and scipy's
     minimum from the PERTURBED start, which on this scene is a different local minimum: the Cauchy loss is
     redescending, so the 1 % outliers (U(+-20 px)) can settle in another basin along another path (scipy
     559.98 vs the oracle's 555.22, variable cost: a worse basin).  Recorded, and asserted to differ.
  2. c1_clean_ba.npz — the same C1 scene without outliers: scipy.optimize.least_squares started from the
     PERTURBED start (independent of the oracle: its own numpy restatement of project.h and the quaternion
     update, finite-difference Jacobian, exact trust-region solves, block Cauchy loss as the smooth residual
     e = r sqrt(rho(s)/s)) reaches the same minimum as the oracle run to tight tolerances; the generator
     asserts the agreement before writing.  The device solver is tested against scipy's minimum.

Usage:  python tests/golden/make_golden.py      (about five minutes: the scipy solves dominate)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from slamgpu.scene import make_config  # noqa: E402


# ---------------------------------------------------------------------------- independent numpy model
def np_project(q, t, k, X):
    """project.h:11-54 vectorised (q Eigen [x,y,z,w], rows)."""
    v = X[:, :3] - t * X[:, 3:4]
    u, w = q[:, :3], q[:, 3:4]
    uv = 2.0 * np.cross(u, v)
    p = v + w * uv + np.cross(u, uv)
    ok = p[:, 2] >= 0.001 * X[:, 3]
    xp, yp = p[:, 0] / p[:, 2], p[:, 1] / p[:, 2]
    r2 = xp * xp + yp * yp
    d = 1 + r2 * (k[:, 0] + r2 * (k[:, 1] + r2 * k[:, 2]))
    return np.stack([k[:, 3] * d * xp + k[:, 5], k[:, 4] * d * yp + k[:, 6]], 1), ok


def np_quat_plus(x, d):
    """ceres::QuaternionParameterization::Plus on Eigen memory (rows)."""
    nd = np.linalg.norm(d, axis=1, keepdims=True)
    s = np.where(nd > 0, np.sin(nd) / np.where(nd > 0, nd, 1), 1.0)
    z = np.concatenate([np.cos(nd), s * d], 1)
    out = np.stack([
        z[:, 0] * x[:, 0] - z[:, 1] * x[:, 1] - z[:, 2] * x[:, 2] - z[:, 3] * x[:, 3],
        z[:, 0] * x[:, 1] + z[:, 1] * x[:, 0] + z[:, 2] * x[:, 3] - z[:, 3] * x[:, 2],
        z[:, 0] * x[:, 2] - z[:, 1] * x[:, 3] + z[:, 2] * x[:, 0] + z[:, 3] * x[:, 1],
        z[:, 0] * x[:, 3] + z[:, 1] * x[:, 2] - z[:, 2] * x[:, 1] + z[:, 3] * x[:, 0]], 1)
    return np.where(nd > 0, out, x)


def _rho_over_s(s, b):
    """Cauchy rho(s)/s = b log(1 + s/b) / s, smooth at s = 0 (limit 1)."""
    small = s < 1e-12 * b
    ss = np.where(small, 1.0, s)
    return np.where(small, 1.0 - s / (2 * b), b * np.log1p(ss / b) / ss)


def scipy_minimum(pa, start=None, max_nfev=500):
    from scipy.optimize import least_squares
    from scipy.sparse import lil_matrix

    q0 = pa.q.reshape(-1, 4)
    t0 = pa.t.reshape(-1, 3)
    X0 = pa.X.reshape(-1, 4)
    k = pa.k.reshape(-1, 7)
    of, op = pa.obs_frame, pa.obs_point
    ff = np.nonzero(pa.frame_rot_free & pa.frame_trans_free)[0]
    fp = np.nonzero(pa.point_free)[0]
    fidx = -np.ones(pa.num_frames, int)
    fidx[ff] = np.arange(len(ff))
    pidx = -np.ones(pa.num_points, int)
    pidx[fp] = np.arange(len(fp))
    var = (fidx[of] >= 0) | (pidx[op] >= 0)
    of_v, op_v, pt_v = of[var], op[var], pa.obs_pt.reshape(-1, 2)[var]
    nF, nP = len(ff), len(fp)
    b = pa.range ** 2

    def unpack(x):
        q = q0.copy(); t = t0.copy(); X = X0.copy()
        xf = x[:6 * nF].reshape(-1, 6)
        q[ff] = np_quat_plus(q0[ff], xf[:, :3])
        t[ff] = xf[:, 3:]
        X[fp, :3] = x[6 * nF:].reshape(-1, 3)
        return q, t, X

    def fun(x):
        q, t, X = unpack(x)
        uv, ok = np_project(q[of_v], t[of_v], k[pa.frame_camera[of_v]], X[op_v])
        rr = uv - pt_v
        s = (rr ** 2).sum(1)
        # block Cauchy loss as a smooth least-squares residual: e = r sqrt(rho(s)/s), 0.5|e|^2 = 0.5 rho(s)
        e = rr * np.sqrt(_rho_over_s(s, b))[:, None]
        ta, tb = t[pa.dist_frame], t[pa.dist_prev]
        r = 0.1 * (np.linalg.norm(ta - tb, axis=1) - pa.dist_target)
        ed = r * np.sqrt(_rho_over_s(r * r, pa.dist_range ** 2))
        return np.concatenate([e.ravel(), ed])

    x0 = np.concatenate([np.concatenate([np.zeros((nF, 3)), t0[ff]], 1).ravel(), X0[fp, :3].ravel()])
    if start is not None:
        # start from another state (q, t, X): rotation offset via the log of q0^-1 q is not needed — use the
        # start state as the new expansion point.
        q0[:], t0[:], X0[:] = (start[0].reshape(-1, 4), start[1].reshape(-1, 3), start[2].reshape(-1, 4))
        x0 = np.concatenate([np.concatenate([np.zeros((nF, 3)), t0[ff]], 1).ravel(), X0[fp, :3].ravel()])
    nobs = len(of_v)
    S = lil_matrix((2 * nobs + len(pa.dist_frame), len(x0)), dtype=int)
    for i, (f, p) in enumerate(zip(of_v, op_v)):
        for row in (2 * i, 2 * i + 1):
            if fidx[f] >= 0:
                S[row, 6 * fidx[f]:6 * fidx[f] + 6] = 1
            if pidx[p] >= 0:
                S[row, 6 * nF + 3 * pidx[p]:6 * nF + 3 * pidx[p] + 3] = 1
    for j, (a, c) in enumerate(zip(pa.dist_frame, pa.dist_prev)):
        for fr in (a, c):
            if fidx[fr] >= 0:
                S[2 * nobs + j, 6 * fidx[fr] + 3:6 * fidx[fr] + 6] = 1
    from scipy.optimize._numdiff import approx_derivative, group_columns
    Sc = S.tocsc()
    groups = group_columns(Sc)

    def jac(x):
        # finite-difference Jacobian over the column groups the sparsity allows, densified so that the trust
        # region subproblem is solved exactly (lsmr's inexact steps stall on this ill-conditioned problem)
        return approx_derivative(fun, x, method="2-point", rel_step=1e-8, sparsity=(Sc, groups)).toarray()

    res = least_squares(fun, x0, jac=jac, method="trf", tr_solver="exact", x_scale="jac", ftol=1e-15,
                        xtol=1e-15, gtol=1e-15, max_nfev=max_nfev)
    print("scipy: status", res.status, "nfev", res.nfev, "cost", res.cost, "start cost", 0.5 * (fun(x0) ** 2).sum())
    q, t, X = unpack(res.x)
    return q, t, X, res.cost, res.nfev


def _evaluate_at(pa, q, t, X):
    ps = pa.copy()
    ps.q[:], ps.t[:], ps.X[:] = q.ravel(), t.ravel(), X.ravel()
    r, cost, nf = oracle.evaluate(ps)
    assert nf == 0
    return ps, r, cost


def _unit_hom(X):
    X = X.reshape(-1, 4)
    return X / np.linalg.norm(X, axis=1, keepdims=True) * np.sign(X[:, 3:])


def make_c1():
    from slamgpu.capi import default_solver_options
    m = make_config("C1")
    pa = oracle.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    inputs = {f"in_{f}": getattr(pa, f) for f in pa.FIELDS}
    inputs.update(in_range=pa.range)
    po = pa.copy()
    s = oracle.solve(po, nthreads=1)
    r, cost_var, nfail = oracle.evaluate(po)
    # (a) local-minimum check: scipy started at the oracle's converged state
    q, t, X, scost, nfev = scipy_minimum(pa.copy(), start=(po.q, po.t, po.X))
    ps, rs, cost_scipy = _evaluate_at(pa, q, t, X)
    # (b) scipy from the perturbed start: another basin of the redescending loss (see the module docstring)
    q2, t2, X2, scost2, nfev2 = scipy_minimum(pa.copy(), max_nfev=200)
    var_oracle = s["final_cost"] - s["fixed_cost"]
    assert scost2 > var_oracle, (scost2, var_oracle)
    # the oracle's first 20 iterations (before the singular-point-block regime), for the device's
    # iteration-for-iteration pin
    p20 = pa.copy()
    s20 = oracle.solve(p20, default_solver_options(max_num_iterations=20), nthreads=1)
    np.savez_compressed(
        os.path.join(HERE, "c1_ba.npz"), **inputs,
        oracle_q=po.q, oracle_t=po.t, oracle_X=po.X, oracle_residuals=r,
        oracle_num_iterations=s["num_iterations"], oracle_num_successful=s["num_successful_steps"],
        oracle_num_invalid=s["num_invalid_steps"],
        oracle_final_cost=s["final_cost"], oracle_initial_cost=s["initial_cost"],
        oracle_fixed_cost=s["fixed_cost"], oracle_termination=s["termination_type"],
        oracle20_q=p20.q, oracle20_t=p20.t, oracle20_X=p20.X, oracle20_final_cost=s20["final_cost"],
        oracle20_num_successful=s20["num_successful_steps"],
        scipy_q=q.ravel(), scipy_t=t.ravel(), scipy_X=X.ravel(), scipy_cost=scost, scipy_nfev=nfev,
        scipy_residuals=rs,
        scipy_start_q=q2.ravel(), scipy_start_t=t2.ravel(), scipy_start_X=X2.ravel(), scipy_start_cost=scost2,
        scipy_start_nfev=nfev2)
    print("C1 oracle:", s)
    print("oracle variable cost %.9f   scipy (from oracle) %.9f (nfev %d)  oracle-eval of scipy point %.9f" %
          (cost_var, scost, nfev, cost_scipy))
    print("scipy from the perturbed start: %.9f (nfev %d) vs oracle %.9f: another local minimum" % (
        scost2, nfev2, var_oracle))
    print("max |t| diff %.3e mm, max |q| diff %.3e" % (np.abs(po.t - ps.t).max(), np.abs(po.q - ps.q).max()))


def make_c1_clean():
    from slamgpu.capi import default_solver_options
    m = make_config("C1", outlier_frac=0.0)
    pa = oracle.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    inputs = {f"in_{f}": getattr(pa, f) for f in pa.FIELDS}
    inputs.update(in_range=pa.range)
    po = pa.copy()
    s = oracle.solve(po, nthreads=1)
    pt = pa.copy()
    tight = default_solver_options(function_tolerance=1e-13, parameter_tolerance=1e-13, max_num_iterations=500)
    st = oracle.solve(pt, tight, nthreads=1)
    _, cost_tight, _ = oracle.evaluate(pt)
    q, t, X, scost, nfev = scipy_minimum(pa.copy(), max_nfev=200)
    ps, rs, cost_scipy = _evaluate_at(pa, q, t, X)
    # the independent minimum and the oracle's agree: the objective (scipy's own cost = the oracle's final
    # cost minus its fixed cost: reprojection + FrameDistance terms of the free blocks), poses and points
    var_tight = st["final_cost"] - st["fixed_cost"]
    assert abs(scost - var_tight) <= 1e-8 * var_tight, (scost, var_tight)
    assert np.abs(ps.t - pt.t).max() < 1e-2
    assert np.abs(ps.q - pt.q).max() < 1e-6
    assert np.abs(_unit_hom(ps.X) - _unit_hom(pt.X)).max() < 1e-5
    np.savez_compressed(
        os.path.join(HERE, "c1_clean_ba.npz"), **inputs,
        oracle_q=po.q, oracle_t=po.t, oracle_X=po.X, oracle_num_iterations=s["num_iterations"],
        oracle_final_cost=s["final_cost"], oracle_fixed_cost=s["fixed_cost"],
        oracle_tight_q=pt.q, oracle_tight_t=pt.t, oracle_tight_X=pt.X, oracle_tight_final_cost=st["final_cost"],
        scipy_q=q.ravel(), scipy_t=t.ravel(), scipy_X=X.ravel(), scipy_cost=scost, scipy_nfev=nfev,
        scipy_oracle_eval_cost=cost_scipy)
    print("C1 clean oracle:", s, "tight:", st["final_cost"], st["num_iterations"])
    print("scipy from the perturbed start %.9f, oracle tight %.9f (variable cost)" % (scost, var_tight))
    print("max |t| diff %.3e mm, max |q| diff %.3e, max unit-X diff %.3e" % (
        np.abs(pt.t - ps.t).max(), np.abs(pt.q - ps.q).max(), np.abs(_unit_hom(ps.X) - _unit_hom(pt.X)).max()))


def main():
    oracle.build()
    which = sys.argv[1:] or ["c1", "c1_clean"]
    if "c1" in which:
        make_c1()
    if "c1_clean" in which:
        make_c1_clean()


if __name__ == "__main__":
    main()
