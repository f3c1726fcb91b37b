"""CPU tests of the bundle-adjustment oracle (oracle/oracle_ba.cpp) — the parity checker itself.

The reference has no tests or fixtures for this path, so the oracle is pinned here by
known-answer projection cases (project.h:11-54), dual-number vs finite-difference Jacobians, the
quaternion update, the committed golden solve and an independent scipy minimum (tests/golden/).
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = np.array([0.0, 0.0, 0.0, 416.0, -416.0, 320.0, 240.0])
GOLDEN = os.path.join(ROOT, "tests", "golden", "c1_ba.npz")


def test_identity_pose_projects_optical_axis_to_principal_point(oracle_lib):
    for z in (1.0, 250.0, 6000.0):
        for lam in (1.0, 0.37, 1e-3):
            X = lam * np.array([0.0, 0.0, z, 1.0])
            uv, ok = oracle_lib.project([0, 0, 0, 1], [0, 0, 0], K, X)
            assert ok[0]
            assert uv[0, 0] == 320.0 and uv[0, 1] == 240.0


def test_homogeneous_scale_invariance(oracle_lib):
    # project.h:33-34: the '/ point[3]' cancels out
    rng = np.random.default_rng(0)
    for _ in range(50):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        t = rng.normal(size=3) * 100
        X = np.array([*rng.normal(size=2) * 500, 3000.0, 1.0]) + np.array([*t, 0.0])
        uv1, ok1 = oracle_lib.project(q, t, K, X)
        uv2, ok2 = oracle_lib.project(q, t, K, 0.123 * X)
        assert ok1[0] == ok2[0]
        if ok1[0]:
            np.testing.assert_allclose(uv1, uv2, rtol=1e-12, atol=1e-9)


def test_behind_camera_threshold(oracle_lib):
    # project.h:27: reject iff p.z < 0.001 * X.w
    _, ok = oracle_lib.project([0, 0, 0, 1], [0, 0, 0], K, [1.0, 1.0, 0.001, 1.0])
    assert ok[0]
    _, ok = oracle_lib.project([0, 0, 0, 1], [0, 0, 0], K, [1.0, 1.0, 0.000999, 1.0])
    assert not ok[0]
    # the same Euclidean point with negative w is rejected by the reference's test
    _, ok = oracle_lib.project([0, 0, 0, 1], [0, 0, 0], K, [0.0, 0.0, -1.0, -1.0])
    assert not ok[0]


def test_radial_distortion_and_intrinsics(oracle_lib):
    k = np.array([0.1, 0.01, 0.001, 400.0, -410.0, 300.0, 200.0])
    x, y = 0.3, -0.2
    uv, ok = oracle_lib.project([0, 0, 0, 1], [0, 0, 0], k, [x, y, 1.0, 1.0])
    r2 = x * x + y * y
    d = 1 + r2 * (0.1 + r2 * (0.01 + r2 * 0.001))
    assert ok[0]
    np.testing.assert_allclose(uv[0], [400 * d * x + 300, -410 * d * y + 200], rtol=1e-14)


def test_eigen_quaternion_rotation_convention(oracle_lib):
    # q = [0, sin(th/2), 0, cos(th/2)] (Eigen [x,y,z,w]) rotates by R_y(th): p = R (X - t)
    th = 0.3
    q = [0.0, np.sin(th / 2), 0.0, np.cos(th / 2)]
    R = np.array([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]])
    t = np.array([10.0, -20.0, 5.0])
    Xw = np.array([100.0, 50.0, 3000.0])
    p = R @ (Xw - t)
    uv, ok = oracle_lib.project(q, t, K, [*Xw, 1.0])
    np.testing.assert_allclose(uv[0], [416 * p[0] / p[2] + 320, -416 * p[1] / p[2] + 240], rtol=1e-12)


def test_dual_number_jacobian_matches_finite_differences(oracle_lib):
    rng = np.random.default_rng(1)
    for _ in range(40):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        t = rng.normal(size=3) * 50
        k = K + np.array([0.02, 0.001, 0.0001, 0, 0, 0, 0]) * rng.normal(size=7)
        Xe = rng.normal(size=3) * 300 + np.array([0, 0, 2500.0])
        X = np.array([*Xe, 1.0]) / np.linalg.norm([*Xe, 1.0])
        ok, uv, J = oracle_lib.project_jet(q, t, k, X)
        if not ok or np.abs(J).max() > 1e9 or np.abs(uv).max() > 1e4:
            continue   # grazing the image plane: finite differences are meaningless there
        x0 = np.concatenate([q, t, k, X])
        Jfd = np.zeros((2, 18))
        for j in range(18):
            h = 1e-6 * max(1.0, abs(x0[j]))
            xp, xm = x0.copy(), x0.copy()
            xp[j] += h
            xm[j] -= h
            up, _ = oracle_lib.project(xp[:4], xp[4:7], xp[7:14], xp[14:])
            um, _ = oracle_lib.project(xm[:4], xm[4:7], xm[7:14], xm[14:])
            Jfd[:, j] = (up[0] - um[0]) / (2 * h)
        np.testing.assert_allclose(J, Jfd, rtol=2e-5, atol=1e-6 * np.abs(J).max())


def test_quaternion_plus_is_a_norm_preserving_retraction(oracle_lib):
    rng = np.random.default_rng(2)
    for _ in range(20):
        x = rng.normal(size=4)
        x /= np.linalg.norm(x)
        d = rng.normal(size=3) * 0.1
        out = oracle_lib.quat_plus(x, d)
        assert abs(np.linalg.norm(out) - 1.0) < 1e-14
        np.testing.assert_array_equal(oracle_lib.quat_plus(x, np.zeros(3)), x)


def test_device_projection_math_matches_dual_numbers_on_host(oracle_lib, tmp_path):
    """slam-robot_amd/csrc/project_math.h (the device math, compiled for the host) vs oracle Jet<18>."""
    exe = tmp_path / "pmc"
    src = os.path.join(ROOT, "tests", "native", "project_math_check.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "slam-robot_amd", "csrc"), src,
                    "-L", os.path.join(ROOT, "oracle"), "-loracle",
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr


def _golden_problem():
    from slamgpu.capi import ProblemArrays
    g = np.load(GOLDEN)
    pa = ProblemArrays(**{f: g[f"in_{f}"] for f in ProblemArrays.FIELDS if f not in
                          ("frame_map_index", "point_map_index")},
                       frame_map_index=g["in_frame_map_index"], point_map_index=g["in_point_map_index"],
                       range_=float(g["in_range"]))
    return pa, g


def test_oracle_reproduces_golden_solve(oracle_lib):
    pa, g = _golden_problem()
    s = oracle_lib.solve(pa, nthreads=1)
    assert s["ok"] == 1 and s["termination"] == "FUNCTION_TOLERANCE"
    assert s["num_iterations"] == int(g["oracle_num_iterations"])
    assert abs(s["final_cost"] - float(g["oracle_final_cost"])) <= 1e-9 * float(g["oracle_final_cost"])
    np.testing.assert_allclose(pa.t, g["oracle_t"], atol=1e-6)
    np.testing.assert_allclose(pa.q, g["oracle_q"], atol=1e-10)
    np.testing.assert_allclose(pa.X, g["oracle_X"], atol=1e-10)


def test_oracle_minimum_matches_independent_scipy_minimum():
    """The committed independent scipy minimum (numpy objective, no oracle code) is within the oracle's
    function-tolerance stop of the oracle's converged state."""
    g = np.load(GOLDEN)
    # objective value agrees: scipy's numpy cost at the oracle point == oracle final cost - fixed cost
    scipy_cost = float(g["scipy_cost"])
    oracle_var = float(g["oracle_final_cost"]) - float(g["oracle_fixed_cost"])
    assert scipy_cost <= oracle_var + 1e-9
    assert (oracle_var - scipy_cost) / oracle_var < 1e-6
    np.testing.assert_allclose(g["scipy_t"], g["oracle_t"], atol=5e-3)      # mm
    np.testing.assert_allclose(g["scipy_q"], g["oracle_q"], atol=1e-6)
    r_o, r_s = g["oracle_residuals"], g["scipy_residuals"]
    assert abs(np.sqrt((r_o ** 2).mean()) - np.sqrt((r_s ** 2).mean())) < 1e-4


def test_scipy_from_perturbed_start_finds_another_basin_on_outlier_scene():
    """On C1 (1 % outliers at U(+-20 px)) scipy started from the PERTURBED start settles in a different, worse
    local minimum of the redescending Cauchy loss than the oracle's (Ceres's) path reaches (559.98 vs 555.22):
    the recorded fact the outlier-free fixture below is there to avoid."""
    g = np.load(GOLDEN)
    oracle_var = float(g["oracle_final_cost"]) - float(g["oracle_fixed_cost"])
    assert float(g["scipy_start_cost"]) > oracle_var * (1 + 1e-4)


CLEAN = os.path.join(ROOT, "tests", "golden", "c1_clean_ba.npz")


def _clean_problem():
    from slamgpu.capi import ProblemArrays
    g = np.load(CLEAN)
    pa = ProblemArrays(**{f: g[f"in_{f}"] for f in ProblemArrays.FIELDS if f not in
                          ("frame_map_index", "point_map_index")},
                       frame_map_index=g["in_frame_map_index"], point_map_index=g["in_point_map_index"],
                       range_=float(g["in_range"]))
    return pa, g


def _unit_hom(X):
    X = np.asarray(X).reshape(-1, 4)
    return X / np.linalg.norm(X, axis=1, keepdims=True) * np.sign(X[:, 3:])


def test_oracle_matches_independent_minimum_from_perturbed_start(oracle_lib):
    """on the outlier-free C1 scene, scipy started from the perturbed start (no oracle code,
    no oracle state) and the oracle solve (re-run here, tight tolerances) reach the same minimum: the
    objective to 1e-8 relative, translations to 1e-2 mm, rotations to 1e-6, points (unit homogeneous) 1e-5."""
    from slamgpu.capi import default_solver_options
    pa, g = _clean_problem()
    tight = default_solver_options(function_tolerance=1e-13, parameter_tolerance=1e-13, max_num_iterations=500)
    s = oracle_lib.solve(pa, tight, nthreads=1)
    var = s["final_cost"] - s["fixed_cost"]
    assert abs(var - float(g["scipy_cost"])) <= 1e-8 * var
    np.testing.assert_allclose(pa.t, g["scipy_t"], atol=1e-2)
    np.testing.assert_allclose(pa.q, g["scipy_q"], atol=1e-6)
    np.testing.assert_allclose(_unit_hom(pa.X), _unit_hom(g["scipy_X"]), atol=1e-5)
    # and the default-tolerance solve is the committed regression pin
    pb, _ = _clean_problem()
    sb = oracle_lib.solve(pb, nthreads=1)
    assert sb["num_iterations"] == int(g["oracle_num_iterations"])
    assert abs(sb["final_cost"] - float(g["oracle_final_cost"])) <= 1e-12 * sb["final_cost"]


def test_oracle_solve_is_deterministic_and_thread_count_stable(oracle_lib):
    from slamgpu.scene import make_config
    m = make_config("C1")
    pa = oracle_lib.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    a, b, c = pa.copy(), pa.copy(), pa.copy()
    sa = oracle_lib.solve(a, nthreads=1)
    sb = oracle_lib.solve(b, nthreads=1)
    sc = oracle_lib.solve(c, nthreads=4)
    assert sa == sb
    np.testing.assert_array_equal(a.X, b.X)
    assert abs(sa["final_cost"] - sc["final_cost"]) < 1e-6 * sa["final_cost"]


def test_reproject_map_semantics(oracle_lib):
    """slam.cpp:523-548: every observation (disabled included); failures keep error = pt and are not
    averaged."""
    from slamgpu.scene import make_config
    m = make_config("C1")
    m.obs_disabled[::7] = 1
    # push one point behind every camera
    m.X[4 * 3:4 * 3 + 4] = [0.0, 0.0, -1.0, 1e-6]
    mean = oracle_lib.reproject_map(m)
    err = m.obs_error.reshape(-1, 2)
    bad = m.obs_point == 3
    np.testing.assert_array_equal(err[bad], m.obs_pt.reshape(-1, 2)[bad])
    assert np.isclose(mean, np.linalg.norm(err[~bad], axis=1).mean(), rtol=1e-12)


def test_reproject_mean_invariant_under_gauge_normalisation(oracle_lib):
    """main.cpp:602-605: ReprojectMap before and after LocalMap::Normalize agree (CHECK_NEAR 0.1);
    Normalize (localmap.cpp:114-155) restated here in numpy: translate frame 0 to the origin, then rotate
    so that frame 0 has identity rotation."""
    from slamgpu.scene import make_config, quat_from_matrix, quat_to_matrix
    m = make_config("C1")
    e1 = oracle_lib.reproject_map(m)
    q = m.q.reshape(-1, 4)
    t = m.t.reshape(-1, 3)
    X = m.X.reshape(-1, 4)
    xl = -t[0].copy()
    t += xl
    X[:, :3] += xl * X[:, 3:4]
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    R0 = quat_to_matrix(q[0])
    inv = np.linalg.inv(R0)
    for f in range(len(q)):
        q[f] = quat_from_matrix(quat_to_matrix(q[f]) @ inv)
        t[f] = R0 @ t[f]
    X[:, :3] = X[:, :3] @ R0.T
    e2 = oracle_lib.reproject_map(m)
    assert abs(e1 - e2) < 0.1
    assert abs(e1 - e2) < 1e-6 * e1


def _numpy_normalize(m):
    """The same gauge change as test_reproject_mean_invariant_under_gauge_normalisation, in numpy."""
    from slamgpu.scene import quat_from_matrix, quat_to_matrix
    q = m.q.reshape(-1, 4)
    t = m.t.reshape(-1, 3)
    X = m.X.reshape(-1, 4)
    xl = -t[0].copy()
    t += xl
    X[:, :3] += xl * X[:, 3:4]
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    R0 = quat_to_matrix(q[0])
    inv = np.linalg.inv(R0)
    for f in range(len(q)):
        q[f] = quat_from_matrix(quat_to_matrix(q[f]) @ inv)
        t[f] = R0 @ t[f]
    X[:, :3] = X[:, :3] @ R0.T


@pytest.mark.parametrize("yaw_deg", [0.0, 30.0, 179.0])
def test_oracle_normalize_restatement(oracle_lib, yaw_deg):
    """oracle_map.cpp's LocalMap::Normalize (localmap.cpp:114-155) against the numpy restatement: frame 0 ends at
    the origin with the identity rotation, the map's reprojection is unchanged (main.cpp:602-605), and a frame
    rotated ~180 deg from frame 0 takes Eigen's largest-diagonal branch of the quaternion-from-matrix."""
    from slamgpu.scene import axis_angle, make_config, quat_from_matrix, quat_to_matrix
    m = make_config("C1")
    # rotate the whole scene (frames and points consistently) so that frame 0 is not the identity
    R = axis_angle(np.deg2rad([10.0, yaw_deg, -5.0]))
    q = m.q.reshape(-1, 4)
    t = m.t.reshape(-1, 3)
    for f in range(len(q)):
        q[f] = quat_from_matrix(quat_to_matrix(q[f]) @ R.T)
        t[f] = R @ t[f] + np.array([100.0, -40.0, 7.0])
    X = m.X.reshape(-1, 4)
    X[:, :3] = X[:, :3] @ R.T + np.array([100.0, -40.0, 7.0]) * X[:, 3:4]
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    if yaw_deg > 90:
        # frame 3 turned ~170 deg from frame 0: R_3 R_0^-1 has a negative trace
        q[3] = quat_from_matrix(axis_angle(np.deg2rad([0.0, 170.0, 0.0])) @ quat_to_matrix(q[0]))
        assert np.trace(quat_to_matrix(q[3]) @ quat_to_matrix(q[0]).T) < 0
    e1 = oracle_lib.reproject_map(m)
    mo, mn = m.copy(), m.copy()
    oracle_lib.normalize(mo)
    _numpy_normalize(mn)
    np.testing.assert_allclose(mo.t, mn.t, rtol=0, atol=1e-9)
    np.testing.assert_allclose(mo.X, mn.X, rtol=0, atol=1e-12)
    # quaternions: the same rotation (q and -q are one rotation; numpy's restatement keeps w >= 0)
    for f in range(mo.num_frames):
        np.testing.assert_allclose(quat_to_matrix(mo.q[4 * f:4 * f + 4]), quat_to_matrix(mn.q[4 * f:4 * f + 4]),
                                   rtol=0, atol=1e-12)
    np.testing.assert_allclose(mo.t[:3], 0.0, atol=1e-12)
    np.testing.assert_allclose(quat_to_matrix(mo.q[:4]), np.eye(3), atol=1e-12)
    e2 = oracle_lib.reproject_map(mo)
    assert abs(e1 - e2) < 0.1 and abs(e1 - e2) <= 1e-9 * e1


def test_oracle_normalize_single_frame_is_untouched(oracle_lib):
    from slamgpu.scene import make_config
    m = make_config("C1")
    one = m.copy()
    one.q, one.t = one.q[:4].copy(), one.t[:3].copy()
    one.frame_camera, one.frame_prev = one.frame_camera[:1].copy(), one.frame_prev[:1].copy()
    keep = one.obs_frame == 0
    one.obs_pt = one.obs_pt.reshape(-1, 2)[keep].reshape(-1).copy()
    one.obs_frame, one.obs_point = one.obs_frame[keep].copy(), one.obs_point[keep].copy()
    one.obs_disabled, one.obs_error = one.obs_disabled[keep].copy(), one.obs_error.reshape(-1, 2)[keep].reshape(-1).copy()
    before = one.copy()
    oracle_lib.normalize(one)
    np.testing.assert_array_equal(one.X, before.X)
    np.testing.assert_array_equal(one.t, before.t)
