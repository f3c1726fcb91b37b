"""GPU parity tests of the device bundle-adjustment solver (libslamgpu.so through the C-ABI) against the
oracle (oracle/oracle_ba.cpp) and the committed golden fixtures.

Tolerances (fp64 device path vs fp64 oracle; the two differ only in summation order and in analytic vs
dual-number derivatives):
  * residual sweep (ReprojectionError at the same state): |dr| <= 1e-9 px, cost rel 1e-12
  * converged solve: final cost rel <= 1e-6, residual RMS within 1e-4 px, translations within 1e-2 mm,
    quaternions within 1e-6 (two LM runs can take different numbers of invalid steps at trust radii
    ~1e15 where the homogeneous point blocks are numerically singular; they converge to the same minimum)
  * behind-camera failure flags, termination types and Slam::iterations()/error() bookkeeping: exact.
"""
import numpy as np
import pytest

from slamgpu import ba
from slamgpu.capi import ProblemArrays, default_solver_options
from slamgpu.scene import make_config, make_scene

pytestmark = pytest.mark.gpu


def _golden():
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "c1_ba.npz"))
    pa = ProblemArrays(**{f: g[f"in_{f}"] for f in ProblemArrays.FIELDS if f not in
                          ("frame_map_index", "point_map_index")},
                       frame_map_index=g["in_frame_map_index"], point_map_index=g["in_point_map_index"],
                       range_=float(g["in_range"]))
    return pa, g


def _solve_both(oracle_lib, pa, options=None, nthreads=1):
    pg, po = pa.copy(), pa.copy()
    g = ba.BundleAdjuster()
    g.load(pg)
    sg = g.solve(options)
    so = oracle_lib.solve(po, options, nthreads=nthreads)
    return pg, sg, po, so


def _assert_same_minimum(oracle_lib, pg, sg, po, so):
    assert sg["ok"] == so["ok"] == 1
    assert sg["sync_timeouts"] == 0
    assert sg["termination"] == so["termination"] or {sg["termination"], so["termination"]} <= {
        "FUNCTION_TOLERANCE", "PARAMETER_TOLERANCE", "GRADIENT_TOLERANCE"}
    assert abs(sg["initial_cost"] - so["initial_cost"]) <= 1e-10 * so["initial_cost"]
    assert abs(sg["fixed_cost"] - so["fixed_cost"]) <= 1e-10 * max(so["fixed_cost"], 1.0)
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"]
    rg, _, fg = oracle_lib.evaluate(pg)
    ro, _, fo = oracle_lib.evaluate(po)
    assert fg == fo == 0
    assert abs(np.sqrt((rg ** 2).mean()) - np.sqrt((ro ** 2).mean())) <= 1e-4
    # a skipped previous frame's translation is constrained only by FrameDistance (|t_a - t_b| = 150): it
    # can sit anywhere on that sphere, so only frames with observations are compared
    seen = np.repeat(pg.frame_rot_free.astype(bool) | ~pg.frame_trans_free.astype(bool), 3)
    np.testing.assert_allclose(pg.t[seen], po.t[seen], atol=1e-2)
    np.testing.assert_allclose(pg.q, po.q, atol=1e-6)


def test_residual_sweep_matches_oracle(gpu_lib, oracle_lib):
    for name in ("C1", "C2"):
        m = make_config(name)
        pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
        g = ba.BundleAdjuster()
        g.load(pa)
        r, cost, nf = g.evaluate()
        ro, co, nfo = oracle_lib.evaluate(pa.copy())
        assert nf == nfo == 0
        np.testing.assert_allclose(r, ro, rtol=0, atol=1e-9)
        assert abs(cost - co) <= 1e-12 * co


def test_c1_first_10_iterations_match_oracle(gpu_lib, oracle_lib):
    """The C1 golden problem's first 10 LM iterations (trust radius up to 6e8) against the oracle, iteration for
    iteration: the same accepted steps, cost to 1e-12 relative, rotations and point directions to 1e-9,
    translations to 1e-9 mm, per-observation residuals to 1e-9 px (measured on MI355X: cost 5e-15, rotations
    5e-15, point directions 3e-13, translations 3e-11 mm, residuals 2.5e-10 px: tools/parity_pins.py)."""
    pa, _ = _golden()
    o = default_solver_options(max_num_iterations=10)
    b = ba.BundleAdjuster()
    pg, po = pa.copy(), pa.copy()
    b.load(pg)
    s = b.solve(o)
    so = oracle_lib.solve(po, o)
    assert s["num_successful_steps"] == so["num_successful_steps"] == 10
    assert abs(s["final_cost"] - so["final_cost"]) <= 1e-12 * so["final_cost"]
    np.testing.assert_allclose(pg.q, po.q, rtol=0, atol=1e-9)
    np.testing.assert_allclose(pg.t, po.t, rtol=0, atol=1e-9)
    # points: their directions to 1e-9 (measured 3e-13); their scale |X| (the gauge of the rank-3 point block)
    # is already drifting by rounding at radius 6e8 (5e-10 relative measured), so X itself is held to 5e-9
    xg, xo = pg.X.reshape(-1, 4), po.X.reshape(-1, 4)
    np.testing.assert_allclose(xg / np.linalg.norm(xg, axis=1, keepdims=True),
                               xo / np.linalg.norm(xo, axis=1, keepdims=True), rtol=0, atol=1e-9)
    np.testing.assert_allclose(pg.X, po.X, rtol=0, atol=5e-9)
    rg, _, _ = oracle_lib.evaluate(pg)
    ro, _, _ = oracle_lib.evaluate(po)
    np.testing.assert_allclose(rg, ro, rtol=0, atol=1e-9)


def test_golden_c1_first_20_iterations(gpu_lib, oracle_lib):
    """The C1 golden's first 20 LM iterations against the committed oracle state: the same accepted steps, and
    the comparison made through gauge-invariant quantities.  By iteration 20 the trust radius is 3.5e13; the
    homogeneous 4x4 point blocks are rank 3 (X and lambda X project alike, project.h:33-34), so the LM damping
    D/radius ~ 1e-14 |V| is below the rounding of V itself and the scale |X| of each point drifts by rounding
    (measured 2.3e-5 relative between the two solvers); the damping metric then moves the other directions at
    the 1e-8 level.  The gauge-invariant figures are the per-observation residuals (what the solve minimises)
    and the cost.  Measured on MI355X (tools/parity_pins.py): cost 2e-10 relative, residuals RMS 2.6e-7 px /
    max 8.7e-6 px, rotations 6.3e-10, translations 2.4e-6 mm; bounds: cost 1e-9, residual RMS 1e-6 px and max
    5e-5 px, rotations 5e-9, translations 1e-5 mm (4x-8x the measured values)."""
    pa, g = _golden()
    b = ba.BundleAdjuster()
    pg = pa.copy()
    b.load(pg)
    s = b.solve(default_solver_options(max_num_iterations=20))
    assert s["num_successful_steps"] == int(g["oracle20_num_successful"]) == 20
    assert abs(s["final_cost"] - float(g["oracle20_final_cost"])) <= 1e-9 * float(g["oracle20_final_cost"])
    np.testing.assert_allclose(pg.q, g["oracle20_q"], rtol=0, atol=5e-9)
    np.testing.assert_allclose(pg.t, g["oracle20_t"], rtol=0, atol=1e-5)   # mm
    po = pa.copy()
    po.q[:], po.t[:], po.X[:] = g["oracle20_q"], g["oracle20_t"], g["oracle20_X"]
    rg, _, fg = oracle_lib.evaluate(pg)
    ro, _, fo = oracle_lib.evaluate(po)
    assert fg == fo == 0
    dr = np.abs(rg - ro)
    assert np.sqrt((dr ** 2).mean()) <= 1e-6 and dr.max() <= 5e-5, (np.sqrt((dr ** 2).mean()), dr.max())
    # point directions (the homogeneous X up to its scale, which is the drifting gauge): 99 % of the points hold
    # the tight per-iteration bound; the rest only the residual bounds above (parity deviations)
    def unit(X):
        X = X.reshape(-1, 4)
        return X / np.linalg.norm(X, axis=1, keepdims=True)
    ddir = np.abs(unit(pg.X) - unit(g["oracle20_X"])).max(axis=1)
    assert np.quantile(ddir, 0.99) <= 1e-6, (np.quantile(ddir, 0.99), ddir.max())


def test_golden_c1_solve(gpu_lib, oracle_lib):
    """The full C1 solve.  The oracle takes 158 iterations: 85 successful, 72 invalid steps at trust radii
    >= 1e15 where the homogeneous point blocks are singular to rounding (test_golden_c1_first_20_iterations), 1
    unsuccessful.  How many invalid steps each solver takes in that regime depends on rounding (measured: the
    device takes 159 with the same 85 successful steps and 73 invalid), so the successful steps are compared
    within 2 and the total within 5, and the minimum to 1e-6 relative cost, 1e-2 mm, 1e-6."""
    pa, g = _golden()
    b = ba.BundleAdjuster()
    pg = pa.copy()
    b.load(pg)
    s = b.solve()
    assert s["ok"] == 1 and s["termination"] == "FUNCTION_TOLERANCE"
    assert abs(s["final_cost"] - float(g["oracle_final_cost"])) <= 1e-6 * float(g["oracle_final_cost"])
    assert abs(s["initial_cost"] - float(g["oracle_initial_cost"])) <= 1e-10 * float(g["oracle_initial_cost"])
    assert abs(s["num_successful_steps"] - int(g["oracle_num_successful"])) <= 2
    assert abs(s["num_iterations"] - int(g["oracle_num_iterations"])) <= 5
    np.testing.assert_allclose(pg.t, g["oracle_t"], atol=1e-2)
    np.testing.assert_allclose(pg.q, g["oracle_q"], atol=1e-6)
    # scipy started at the oracle's minimum stays there (local-minimum check)
    np.testing.assert_allclose(pg.t, g["scipy_t"], atol=1e-2)


def test_golden_c1_clean_matches_independent_minimum(gpu_lib):
    """the outlier-free C1 scene solved on the device (tight tolerances) reaches the minimum
    scipy found from the perturbed start with no oracle code (tests/golden/make_golden.py): objective to 1e-8
    relative, translations 1e-2 mm, rotations 1e-6, points (unit homogeneous) 1e-5."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "c1_clean_ba.npz"))
    pa = ProblemArrays(**{f: g[f"in_{f}"] for f in ProblemArrays.FIELDS if f not in
                          ("frame_map_index", "point_map_index")},
                       frame_map_index=g["in_frame_map_index"], point_map_index=g["in_point_map_index"],
                       range_=float(g["in_range"]))
    b = ba.BundleAdjuster()
    pg = pa.copy()
    b.load(pg)
    s = b.solve(default_solver_options(function_tolerance=1e-13, parameter_tolerance=1e-13,
                                       max_num_iterations=500))
    assert s["ok"] == 1 and s["sync_timeouts"] == 0
    var = s["final_cost"] - s["fixed_cost"]
    assert abs(var - float(g["scipy_cost"])) <= 1e-8 * var
    np.testing.assert_allclose(pg.t, g["scipy_t"], atol=1e-2)
    np.testing.assert_allclose(pg.q, g["scipy_q"], atol=1e-6)
    Xg = pg.X.reshape(-1, 4)
    Xs = g["scipy_X"].reshape(-1, 4)
    unit = lambda X: X / np.linalg.norm(X, axis=1, keepdims=True) * np.sign(X[:, 3:])  # noqa: E731
    np.testing.assert_allclose(unit(Xg), unit(Xs), atol=1e-5)


@pytest.mark.parametrize("seed", [1, 3, 4, 7])
def test_c1_sized_solves_match_oracle(gpu_lib, oracle_lib, seed):
    m = make_scene(num_frames=10, num_points=500, seed=seed, run_max=14)
    pa = ba.problem_from_map_frames(m, 8, 10, 2.0)
    _assert_same_minimum(oracle_lib, *_solve_both(oracle_lib, pa))


def test_c2_solve_matches_oracle_iteration_for_iteration(gpu_lib, oracle_lib):
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    pg, sg, po, so = _solve_both(oracle_lib, pa, nthreads=8)
    _assert_same_minimum(oracle_lib, pg, sg, po, so)
    # no invalid steps on this scene: the two LM trajectories coincide
    assert sg["num_iterations"] == so["num_iterations"]
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]


def test_c5_first_iterations_match_oracle(gpu_lib, oracle_lib):
    """BASELINE config 5 on one GPU: 200 keyframes / ~194k landmarks / ~1.95M observations,
    SolveFrames(map, 198, 200, 2.0) (slam.cpp:417-443).  The reduced camera system is n = 1188 (198 free
    frames) with a co-visibility band of <= 8 16-wide tiles, factored by the tiled band Cholesky.  Three LM
    iterations against the oracle's dense solve, iteration for iteration: the same accepted steps, cost to
    1e-9 relative, rotations to 1e-9, translations to 1e-6 mm, points to 1e-9."""
    import os
    m = make_config("C5")
    assert m.num_frames == 200 and m.num_points > 190000 and m.num_obs > 1.9e6
    pa = ba.problem_from_map_frames(m, 198, 200, 2.0)
    o = default_solver_options(max_num_iterations=3)
    pg, po = pa.copy(), pa.copy()
    g = ba.BundleAdjuster()
    g.load(pg)
    info = g.info()
    assert info["n"] == 6 * 198 and info["band_tiles"] <= 8
    assert info["cholesky"].startswith("tiled band")
    assert info["lin_waves"] == 1   # ~10 k Jacobian-sweep chunks fill the chip with one wave each
    sg = g.solve(o)
    so = oracle_lib.solve(po, o, nthreads=min(16, os.cpu_count() or 1))
    assert sg["ok"] == so["ok"] == 1 and sg["sync_timeouts"] == 0
    assert sg["num_iterations"] == so["num_iterations"] == 4
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sg["initial_cost"] - so["initial_cost"]) <= 1e-10 * so["initial_cost"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]
    np.testing.assert_allclose(pg.q, po.q, rtol=0, atol=1e-9)
    np.testing.assert_allclose(pg.t, po.t, rtol=0, atol=1e-6)
    np.testing.assert_allclose(pg.X, po.X, rtol=0, atol=1e-9)


def test_wide_points_and_edge_structure(gpu_lib, oracle_lib):
    """Points seen over > 24 free frames (global-atomic 'wide' path), constant points, a skipped previous
    frame whose translation is freed by FrameDistance, disabled observations and unusable points."""
    m = make_scene(num_frames=40, num_points=400, seed=21, run_max=40)
    rng = np.random.default_rng(0)
    m.obs_disabled[rng.random(m.num_obs) < 0.05] = 1
    m.obs_disabled[m.obs_frame == 30] = 1
    m.point_uncertainty[:] = 1.0
    # this scene has weakly constrained directions (a skipped frame's translation on the FrameDistance
    # sphere, thin point tracks): with the default function tolerance the LM stops at a trajectory-dependent
    # point along them, so both solvers run to tight tolerances here and must meet at the same minimum
    tight = default_solver_options(function_tolerance=1e-13, parameter_tolerance=1e-13, max_num_iterations=200)
    for solve, present in ((38, 40), (9, 14), (20, 40)):
        pa = ba.problem_from_map_frames(m, solve, present, 2.0)
        _assert_same_minimum(oracle_lib, *_solve_both(oracle_lib, pa, tight))


@pytest.mark.parametrize("solve,present", [(38, 40), (9, 14), (20, 40)])
def test_wide_scene_first_steps_match_oracle(gpu_lib, oracle_lib, solve, present):
    """Two LM iterations on the edge-structure scene: the device step (assembly of blockdiag(U), FrameDistance
    blocks and damping into S, banded Cholesky, back substitution) matches the oracle's dense solve."""
    m = make_scene(num_frames=40, num_points=400, seed=21, run_max=40)
    rng = np.random.default_rng(0)
    m.obs_disabled[rng.random(m.num_obs) < 0.05] = 1
    m.obs_disabled[m.obs_frame == 30] = 1
    m.point_uncertainty[:] = 1.0
    pa = ba.problem_from_map_frames(m, solve, present, 2.0)
    o = default_solver_options(max_num_iterations=2)
    pg, sg, po, so = _solve_both(oracle_lib, pa, o)
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]
    np.testing.assert_allclose(pg.t, po.t, atol=1e-6)
    np.testing.assert_allclose(pg.q, po.q, atol=1e-9)


def test_behind_camera_at_start_is_a_numerical_failure(gpu_lib, oracle_lib):
    m = make_config("C1")
    pa = ba.problem_from_map_frames(m, 8, 10, 2.0)
    # put a free point behind the cameras it is observed from
    i = int(np.nonzero(pa.point_free)[0][0])
    pa.X[4 * i:4 * i + 4] = [0.0, 0.0, -1.0, 1e-4]
    pg, sg, po, so = _solve_both(oracle_lib, pa)
    assert sg["ok"] == so["ok"] == 0
    assert sg["termination"] == so["termination"] == "NUMERICAL_FAILURE"


def test_max_iterations_bookkeeping(gpu_lib, oracle_lib):
    m = make_config("C1")
    pa = ba.problem_from_map_frames(m, 8, 10, 2.0)
    o = default_solver_options(max_num_iterations=3)
    pg, sg, po, so = _solve_both(oracle_lib, pa, o)
    assert sg["termination"] == so["termination"] == "NO_CONVERGENCE"
    assert sg["num_iterations"] == so["num_iterations"] == 4      # iteration 0 + 3
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]
    np.testing.assert_allclose(pg.X, po.X, atol=1e-9)


def test_benchmark_mode_runs_exact_iteration_count(gpu_lib):
    m = make_config("C1")
    pa = ba.problem_from_map_frames(m, 8, 10, 2.0)
    g = ba.BundleAdjuster()
    g.load(pa)
    g.begin(default_solver_options(max_num_iterations=10 ** 6, disable_termination=1))
    g.iterate(37)
    g.sync()
    s = g.summary()
    assert s["num_lm_iterations"] == 37
    assert s["ok"] == 1


def test_slam_facade_matches_reference_call_sequence(gpu_lib, oracle_lib):
    """main.cpp:580-605: SolveFrames(2,5), ReprojectMap, SolveFrames(10,20), ReprojectMap — the device Slam
    and the oracle's Slam restatement on identical map copies."""
    m = make_scene(num_frames=24, num_points=1500, seed=5, run_max=10)
    mg, mo = m.copy(), m.copy()
    slam = ba.Slam()
    it_o, err_o = 0, 0.0
    for solve, present in ((2, 5), (10, 20)):
        ok_g = slam.SolveFrames(mg, solve, present, 2.0)
        ok_o, so = oracle_lib.slam_solve_frames(mo, solve, present, 2.0)
        assert ok_g == ok_o
        it_o += so["num_iterations"]
        err_o = so["final_cost"]
        eg = slam.ReprojectMap(mg)
        eo = oracle_lib.reproject_map(mo)
        assert abs(eg - eo) <= 1e-6 * eo
        np.testing.assert_allclose(mg.t, mo.t, atol=1e-2)
    assert abs(slam.error() - err_o) <= 1e-6 * err_o
    assert abs(slam.iterations() - it_o) <= 20
    assert slam.SolveFramePose(None, None) is False


def test_reproject_map_matches_oracle(gpu_lib, oracle_lib):
    m = make_config("C1")
    m.obs_disabled[::5] = 1
    m.X[4 * 7:4 * 7 + 4] = [0.0, 0.0, -1.0, 1e-6]    # point 7 fails to project everywhere
    mg, mo = m.copy(), m.copy()
    eg = ba.Slam().ReprojectMap(mg)
    eo = oracle_lib.reproject_map(mo)
    assert abs(eg - eo) <= 1e-12 * eo
    np.testing.assert_allclose(mg.obs_error, mo.obs_error, atol=1e-9)
    bad = np.repeat(m.obs_point == 7, 2)
    np.testing.assert_array_equal(mg.obs_error[bad], m.obs_pt[bad])


def test_slam_too_few_frames_returns_false(gpu_lib):
    m = make_config("C1")
    slam = ba.Slam()
    assert slam.SolveFrames(m, 1, 1, 2.0) is False
    assert slam.iterations() == 0


def test_packed_band_exchange_is_exact(gpu_lib, monkeypatch):
    """The landmark-shard exchange packs the band of S (per panel: rows of the panel, columns up to its band
    end) and the rhs into one buffer for the all-reduce and unpacks it afterwards.  Forced on
    one GPU (SG_PACK_S), the pack/unpack round trip must leave the solve unchanged.  It is a copy, and the
    device chain is deterministic at C2 (k_schur sums each window tile in MFMA accumulators in point order;
    no point is wide enough for the global-atomic k_schur_wide path), so the two solves agree bit for bit."""
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    out = []
    for force in (False, True):
        if force:
            monkeypatch.setenv("SG_PACK_S", "1")
        p = pa.copy()
        g = ba.BundleAdjuster()
        g.load(p)
        s = g.solve(default_solver_options(max_num_iterations=6))
        out.append((s, p))
        g.close()
    (s0, p0), (s1, p1) = out
    assert s0 == s1
    np.testing.assert_array_equal(p0.q, p1.q)
    np.testing.assert_array_equal(p0.t, p1.t)
    np.testing.assert_array_equal(p0.X, p1.X)



@pytest.mark.parametrize("frames,points", [(36, 8000), (40, 9000), (50, None)])
def test_dissected_band_matches_one_workgroup(gpu_lib, monkeypatch, frames, points):
    """The tiled Cholesky factors the band from both ends at once (k_chol_tiles: a second workgroup factors
    the bottom tile rows of the index-reversed system and hands its separator contribution over; DESIGN.md
    4).  Against the one-workgroup factorisation (SG_CHOL_SPLIT=0) the solve must be the same up to rounding
    (the separator sums in another order): same steps, cost rel 1e-12, poses 1e-10 — with the fixed 7-row
    separator (SG_CHOL_SEP=7: n = 204 -> 13 tile rows, 2 bottom; 228 -> 15, 3; C2's 288 -> 18, 4) and with the
    separator sized to the band (round 6: C2's rows are 6-7 tiles wide, so 5 rows and 6 bottom).  By default
    k_S_reduce factors the first diagonal tile (Z_0) for k_chol_tiles; "own_d0" (SG_CHOL_ZPRE=0) has the Cholesky
    factor it itself, as before round 6 (z_0 then comes from the augmented column, not Z_0 y_0: rounding only)."""
    if points is None:
        m = make_config("C2")
    else:
        m = make_scene(num_frames=frames, num_points=points, seed=5, run_max=14)
    pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    nt = (6 * (m.num_frames - 2) + 15) // 16
    out = []
    for mode in ("one", "sep7", "adaptive", "own_d0"):
        monkeypatch.setenv("SG_CHOL_SPLIT", "0" if mode == "one" else "1")
        monkeypatch.setenv("SG_CHOL_SEP", "7" if mode == "sep7" else "0")
        monkeypatch.setenv("SG_CHOL_ZPRE", "0" if mode == "own_d0" else "1")
        p = pa.copy()
        g = ba.BundleAdjuster()
        g.load(p)
        info = g.info()
        assert info["cholesky"].startswith("tiled band")
        if mode == "one":
            assert info["cholesky_split"] == 0
        elif mode == "sep7":
            assert info["cholesky_split"] == (nt - 9) // 2 and info["cholesky_separator"] == 7
        else:
            ns, nd = info["cholesky_separator"], info["cholesky_split"]
            assert 1 <= ns <= 7 and nd >= 2 and nt - nd - ns >= 1
            if points is None:
                assert (ns, nd) == (5, 6)
        s = g.solve(default_solver_options(max_num_iterations=8))
        out.append((s, p))
        g.close()
    s0, p0 = out[0]
    for s1, p1 in out[1:]:
        assert s0["ok"] == s1["ok"] == 1
        assert s0["sync_timeouts"] == s1["sync_timeouts"] == 0
        assert s0["num_iterations"] == s1["num_iterations"]
        assert s0["num_successful_steps"] == s1["num_successful_steps"]
        assert abs(s0["final_cost"] - s1["final_cost"]) <= 1e-12 * s0["final_cost"]
        np.testing.assert_allclose(p0.q, p1.q, rtol=0, atol=1e-10)
        np.testing.assert_allclose(p0.t, p1.t, rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(p0.X, p1.X, rtol=1e-9, atol=1e-10)

def _intrinsics_scene(seed=1):
    """C1-sized scene whose intrinsics start off the generating camera (focal +0.4 %, principal point +1.5 px,
    a little radial distortion), so SolveAllFrames(..., solve_cameras=true) has intrinsics to recover."""
    m = make_scene(num_frames=10, num_points=500, seed=seed, run_max=14)
    for c in range(len(m.k) // 7):
        k = m.k[7 * c:7 * c + 7]
        k[0] += 2e-3
        k[3] *= 1.004
        k[4] *= 1.004
        k[5] += 1.5
        k[6] -= 1.5
    return m


def test_free_intrinsics_first_steps_match_oracle(gpu_lib, oracle_lib):
    """Two LM iterations with the intrinsics free (slam.cpp:447-480): the k columns of the reduced system
    (J_k terms, CameraStabilization, their point elimination) and the candidate intrinsics match the
    oracle's dense solve."""
    m = _intrinsics_scene()
    pa = ba.problem_from_map_all(m, 2.0, solve_cameras=True)
    assert pa.cameras_free == 1
    o = default_solver_options(max_num_iterations=2, function_tolerance=1e-9)
    pg, sg, po, so = _solve_both(oracle_lib, pa, o)
    assert sg["ok"] == so["ok"] == 1
    assert abs(sg["initial_cost"] - so["initial_cost"]) <= 1e-10 * so["initial_cost"]
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-8 * so["final_cost"]
    np.testing.assert_allclose(pg.k, po.k, rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(pg.t, po.t, atol=1e-5)


def test_free_intrinsics_solve_matches_oracle(gpu_lib, oracle_lib):
    """A full SolveAllFrames(..., true) solve (fine tolerance 1e-9): same minimum as the oracle.  All frames are
    free here (7-DoF gauge), so poses are compared through the residuals; the intrinsics are gauge-invariant."""
    m = _intrinsics_scene(seed=3)
    pa = ba.problem_from_map_all(m, 2.0, solve_cameras=True)
    o = default_solver_options(function_tolerance=1e-9)
    pg, sg, po, so = _solve_both(oracle_lib, pa, o)
    assert sg["ok"] == so["ok"] == 1
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"]
    rg, _, fg = oracle_lib.evaluate(pg)
    ro, _, fo = oracle_lib.evaluate(po)
    assert fg == fo == 0
    assert abs(np.sqrt((rg ** 2).mean()) - np.sqrt((ro ** 2).mean())) <= 1e-4
    np.testing.assert_allclose(pg.k, po.k, rtol=1e-5, atol=1e-6)


def test_free_intrinsics_one_camera_matches_oracle(gpu_lib, oracle_lib):
    """One camera (nk = 7): the bordered band solve's 16-wide border tile is half padding (identity on the
    padded diagonal, zero coupling); two LM iterations against the oracle as in the two-camera test."""
    m = _intrinsics_scene(seed=5)
    m.frame_camera[:] = 0
    m.k = m.k[:7].copy()
    pa = ba.problem_from_map_all(m, 2.0, solve_cameras=True)
    o = default_solver_options(max_num_iterations=2, function_tolerance=1e-9)
    g = ba.BundleAdjuster()
    g.load(pa.copy())
    info = g.info()
    g.close()
    assert info["cholesky_path"] == 4 and info["n"] == info["num_blocks"] * 6 + 7, info
    pg, sg, po, so = _solve_both(oracle_lib, pa, o)
    assert sg["ok"] == so["ok"] == 1
    assert abs(sg["initial_cost"] - so["initial_cost"]) <= 1e-10 * so["initial_cost"]
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-8 * so["final_cost"]
    np.testing.assert_allclose(pg.k, po.k, rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(pg.t, po.t, atol=1e-5)


def test_free_intrinsics_three_cameras_take_the_arrowhead_path(gpu_lib, oracle_lib):
    """Three cameras (nk = 21 > 16): the border does not fit one tile, so the load takes the arrowhead
    k_cholesky_global; two LM iterations against the oracle."""
    m = _intrinsics_scene(seed=6)
    m.frame_camera[:] = np.arange(len(m.frame_camera), dtype=np.int32) % 3
    m.k = np.concatenate([m.k, m.k[:7]])
    pa = ba.problem_from_map_all(m, 2.0, solve_cameras=True)
    o = default_solver_options(max_num_iterations=2, function_tolerance=1e-9)
    g = ba.BundleAdjuster()
    g.load(pa.copy())
    info = g.info()
    g.close()
    assert info["cholesky_path"] in (1, 2, 3) and info["n"] == info["num_blocks"] * 6 + 21, info
    pg, sg, po, so = _solve_both(oracle_lib, pa, o)
    assert sg["ok"] == so["ok"] == 1
    assert abs(sg["initial_cost"] - so["initial_cost"]) <= 1e-10 * so["initial_cost"]
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-8 * so["final_cost"]
    np.testing.assert_allclose(pg.k, po.k, rtol=1e-7, atol=1e-9)


def test_slam_solve_all_frames_with_cameras(gpu_lib, oracle_lib):
    """Slam::SolveAllFrames(map, 2.0, true) through the facade writes the solved intrinsics back to the map."""
    m = _intrinsics_scene(seed=4)
    mg, mo = m.copy(), m.copy()
    slam = ba.Slam()
    ok_g = slam.SolveAllFrames(mg, 2.0, True)
    ok_o, so = oracle_lib.slam_solve_all_frames(mo, 2.0, True)
    assert ok_g == ok_o is True
    assert abs(slam.error() - so["final_cost"]) <= 1e-6 * so["final_cost"]
    np.testing.assert_allclose(mg.k, mo.k, rtol=1e-5, atol=1e-6)
    assert not np.allclose(mg.k, m.k)


def test_solve_is_bitwise_reproducible(gpu_lib):
    """Two C2 solves on fresh handles agree bit for bit: k_schur sums every window tile in MFMA accumulators
    in point order, the camera and Schur partials are reduced in host-fixed order, and the in-wave LDS
    accumulation of k_linearize is serialised by its per-block lists (only k_schur_wide, for points wider
    than a segment window, uses global atomics; C2 has none)."""
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    out = []
    for _ in range(2):
        p = pa.copy()
        g = ba.BundleAdjuster()
        g.load(p)
        out.append((g.solve(), p))
        g.close()
    (s0, p0), (s1, p1) = out
    assert s0 == s1
    np.testing.assert_array_equal(p0.q, p1.q)
    np.testing.assert_array_equal(p0.t, p1.t)
    np.testing.assert_array_equal(p0.X, p1.X)


def test_problem_without_frame_distance(gpu_lib, oracle_lib):
    """num_dist = 0 (no frame has a presented previous frame): k_cam_finalize's FrameDistance prefetch must not
    touch the (padded) empty pair arrays, and the solve matches the oracle."""
    m = make_config("C1")
    pa = ba.problem_from_map_frames(m, 8, 10, 2.0)
    pa.dist_frame = np.zeros(0, np.int32)
    pa.dist_prev = np.zeros(0, np.int32)
    pg, sg, po, so = _solve_both(oracle_lib, pa, default_solver_options(max_num_iterations=4))
    assert sg["ok"] == so["ok"] == 1
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]
    np.testing.assert_allclose(pg.t, po.t, rtol=0, atol=1e-6)


def test_cholesky_handoff_timeout_is_reported(gpu_lib, monkeypatch):
    """The dissected Cholesky's separator wait is bounded.  Forced to time out (SG_CHOL_FORCE_TIMEOUT: the
    bottom workgroup sleeps ~2 ms, the top polls 256 times), the solve must end with DEVICE_TIMEOUT, ok = 0 and
    a non-zero sync_timeouts count (slam.cpp:520: the caller sees the failure) instead of silently rejecting
    the step; without the knob the same solve reports zero time-outs."""
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    o = default_solver_options(max_num_iterations=3)
    g = ba.BundleAdjuster()
    g.load(pa.copy())
    assert g.info()["cholesky_split"] > 0
    s = g.solve(o)
    assert s["ok"] == 1 and s["sync_timeouts"] == 0
    g.close()
    monkeypatch.setenv("SG_CHOL_FORCE_TIMEOUT", "1")
    g = ba.BundleAdjuster()
    g.load(pa.copy())
    s = g.solve(o)
    g.close()
    assert s["termination"] == "DEVICE_TIMEOUT" and s["ok"] == 0
    assert s["sync_timeouts"] >= 1


@pytest.mark.parametrize("path", ["border", "staged", "unstaged"])
def test_free_intrinsics_c2_global_cholesky_matches_oracle(gpu_lib, oracle_lib, monkeypatch, path):
    """SolveAllFrames(C2 map, 2.0, true) (slam.cpp:447-480) at the size where the free-intrinsics path runs its
    global-memory pieces: n = 314 > kCholWS, S is an arrowhead (the frame band, dense through the 14 intrinsics
    columns), and 48 free frame blocks > kIntrWin = 32, so k_intr_lin / k_intr_schur take their out-of-window
    global-atomic branches.  The default factors it as a bordered band (k_chol_tiles on the 19 frame tile rows,
    k_chol_border for the intrinsics: forward chain, 14 x 14 Schur complement, band back substitution);
    SG_CHOL_BORDER=0 takes k_cholesky_global (arrowhead trailing update, MFMA tiles; with and without the
    LDS-staged panel rows, SG_CHOL_GSTAGE=0).  Three LM iterations against the oracle's dense solve: the same
    steps, cost to 1e-8 relative, intrinsics to 1e-7, translations to 1e-5 mm."""
    import os
    if path != "border":
        monkeypatch.setenv("SG_CHOL_BORDER", "0")
        monkeypatch.setenv("SG_CHOL_GSTAGE", "1" if path == "staged" else "0")
    m = make_config("C2")
    for c in range(len(m.k) // 7):
        k = m.k[7 * c:7 * c + 7]
        k[3] *= 1.002
        k[4] *= 1.002
        k[5] += 1.0
    pa = ba.problem_from_map_all(m, 2.0, solve_cameras=True)
    pg, po = pa.copy(), pa.copy()
    g = ba.BundleAdjuster()
    g.load(pg)
    info = g.info()
    assert info["n"] > 128 and info["num_blocks"] > 32
    assert info["cholesky_path"] == {"border": 4, "staged": 2, "unstaged": 3}[path], info
    o = default_solver_options(max_num_iterations=3)
    sg = g.solve(o)
    so = oracle_lib.solve(po, o, nthreads=min(16, os.cpu_count() or 1))
    assert sg["ok"] == so["ok"] == 1 and sg["sync_timeouts"] == 0
    assert sg["num_iterations"] == so["num_iterations"]
    assert sg["num_successful_steps"] == so["num_successful_steps"] >= 2
    assert abs(sg["initial_cost"] - so["initial_cost"]) <= 1e-10 * so["initial_cost"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-8 * so["final_cost"]
    np.testing.assert_allclose(pg.k, po.k, rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(pg.t, po.t, atol=1e-5)


def _solve_env(pa, env, monkeypatch, options=None, bench=None):
    """Solve pa.copy() on a fresh handle with the environment switches env; bench = (W, K): begin with
    termination off and always-linearize, W + K iterations, download (the benchmark's regime)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    p = pa.copy()
    g = ba.BundleAdjuster()
    g.load(p)
    if bench is None:
        s = g.solve(options)
    else:
        g.begin(default_solver_options(max_num_iterations=10 ** 6, disable_termination=1, always_linearize=1))
        g.iterate(bench[0])
        g.iterate(bench[1])
        g.sync()
        s = g.summary()
        g.download()
    g.close()
    for k in env:
        monkeypatch.delenv(k, raising=False)
    return s, p


@pytest.mark.parametrize("regime", ["solve", "bench"])
def test_speculative_linearization_matches_two_pass_chain(gpu_lib, monkeypatch, regime):
    """k_update_lin (the candidate pass linearizes at the candidate into the other slot; k_linearize only in a
    solve's first iteration) against k_point_update + k_linearize every iteration (SG_SPEC=0) on C2.  The J
    records, point blocks and camera partials are the same arithmetic at the same point in the same order; the
    one difference is the candidate cost the decision compares, taken from the linearization's forward value
    instead of a separate Project() (the same formula, contracted differently by the compiler: a rounding-level
    difference in the trust-region ratio).  A full solve from the perturbed start: the same steps, cost 1e-12
    relative, poses 1e-10 / 1e-6 mm, point directions 1e-9.  60 iterations of the benchmark regime (termination
    off, a rejected step re-reduces the current slot instead of re-linearizing), past convergence into rejected
    and invalid steps, where the trust radius follows rounding: the same minimum (cost 2e-9, poses 1e-8 /
    1e-5 mm)."""
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    bench = None if regime == "solve" else (20, 40)
    s0, p0 = _solve_env(pa, {"SG_SPEC": "0"}, monkeypatch, bench=bench)
    s1, p1 = _solve_env(pa, {}, monkeypatch, bench=bench)
    assert s0["ok"] == s1["ok"] == 1 and s1["sync_timeouts"] == 0
    if bench is None:
        for k in ("num_iterations", "num_successful_steps", "num_unsuccessful_steps", "termination"):
            assert s0[k] == s1[k], k
        assert abs(s0["final_cost"] - s1["final_cost"]) <= 1e-12 * s0["final_cost"]
        np.testing.assert_allclose(p1.q, p0.q, rtol=0, atol=1e-10)
        np.testing.assert_allclose(p1.t, p0.t, rtol=0, atol=1e-6)
        # points up to their homogeneous scale (the rank-3 gauge of the point blocks drifts by rounding: measured
        # 7e-7 in X itself at the converged state)
        x0, x1 = p0.X.reshape(-1, 4), p1.X.reshape(-1, 4)
        np.testing.assert_allclose(x1 / np.linalg.norm(x1, axis=1, keepdims=True),
                                   x0 / np.linalg.norm(x0, axis=1, keepdims=True), rtol=0, atol=1e-9)
    else:
        assert s1["num_unsuccessful_steps"] > 0 and s1["num_lm_iterations"] == s0["num_lm_iterations"] == 60
        # measured 6e-11 with the 7-row separator, 7.2e-10 with C2's 5-row one (round 6): past convergence the
        # accept / reject sequence follows rounding, so the two chains end at the same minimum by different paths
        assert abs(s0["final_cost"] - s1["final_cost"]) <= 2e-9 * s0["final_cost"]
        np.testing.assert_allclose(p1.q, p0.q, rtol=0, atol=1e-8)
        np.testing.assert_allclose(p1.t, p0.t, rtol=0, atol=1e-5)


@pytest.mark.parametrize("spec", ["1", "0"])
def test_two_wave_chunks_match_one_wave(gpu_lib, monkeypatch, spec):
    """k_linearize / k_update_lin with a chunk's rounds split over two waves (the default at C2: 2 nlin waves
    fit the chip) against one wave per chunk (SG_LIN_WAVES=1, config 5's choice).  The two waves' camera
    partials and chunk scalars are summed once more at the end, so the sums differ by rounding: the same steps,
    cost 1e-12 relative, poses 1e-10 / 1e-6 mm; the speculative and two-pass chains agree on each split."""
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    g = ba.BundleAdjuster()
    g.load(pa.copy())
    assert g.info()["lin_waves"] == 2
    g.close()
    s1, p1 = _solve_env(pa, {"SG_LIN_WAVES": "1", "SG_SPEC": spec}, monkeypatch)
    s2, p2 = _solve_env(pa, {"SG_LIN_WAVES": "2", "SG_SPEC": spec}, monkeypatch)
    assert s1["ok"] == s2["ok"] == 1 and s2["sync_timeouts"] == 0
    for k in ("num_iterations", "num_successful_steps", "num_unsuccessful_steps", "termination"):
        assert s1[k] == s2[k], k
    assert abs(s1["final_cost"] - s2["final_cost"]) <= 1e-12 * s1["final_cost"]
    np.testing.assert_allclose(p2.q, p1.q, rtol=0, atol=1e-10)
    np.testing.assert_allclose(p2.t, p1.t, rtol=0, atol=1e-6)


def test_speculative_solve_is_bitwise_reproducible_with_rejections(gpu_lib, monkeypatch):
    """The speculative chain in the benchmark regime past convergence (rejected and invalid steps: the current
    slot is re-reduced, the candidate slot overwritten) is deterministic: two fresh handles agree bit for bit."""
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    s0, p0 = _solve_env(pa, {}, monkeypatch, bench=(20, 40))
    s1, p1 = _solve_env(pa, {}, monkeypatch, bench=(20, 40))
    assert s0["num_unsuccessful_steps"] > 0
    assert s0 == s1
    np.testing.assert_array_equal(p0.q, p1.q)
    np.testing.assert_array_equal(p0.X, p1.X)


def test_speculative_linearization_wide_chunks(gpu_lib, oracle_lib, monkeypatch):
    """Points with more than 64 observations or wider than 24 blocks (k_linearize's wide chunks: one point over
    several rounds, camera terms by global atomics into the slotted cam_wide) on the edge-structure scene, with
    tight tolerances: speculative and non-speculative solves agree to rounding (the wide
    chunks' atomics sum in arrival order) and match the oracle's minimum."""
    m = make_scene(num_frames=40, num_points=400, seed=21, run_max=40)
    rng = np.random.default_rng(0)
    m.obs_disabled[rng.random(m.num_obs) < 0.05] = 1
    m.point_uncertainty[:] = 1.0
    pa = ba.problem_from_map_frames(m, 38, 40, 2.0)
    tight = default_solver_options(function_tolerance=1e-13, parameter_tolerance=1e-13, max_num_iterations=200)
    s0, p0 = _solve_env(pa, {"SG_SPEC": "0"}, monkeypatch, options=tight)
    s1, p1 = _solve_env(pa, {}, monkeypatch, options=tight)
    assert s1["ok"] == 1
    assert abs(s0["final_cost"] - s1["final_cost"]) <= 1e-10 * s0["final_cost"]
    np.testing.assert_allclose(p1.q, p0.q, atol=1e-7)
    po = pa.copy()
    so = oracle_lib.solve(po, tight)
    _assert_same_minimum(oracle_lib, p1, s1, po, so)


def test_merged_exchange_chain_on_one_rank(gpu_lib, monkeypatch):
    """The landmark shards' merged exchange chain forced on one rank (SG_XCHG_MERGE=force: k_S_reduce assembles
    the rank's own camera blocks and FrameDistance terms without the damping, S travels packed with the camera
    gradient / diagonal / cost scalars in its tail, k_cam_finalize mode 2 does the bookkeeping and adds the
    damping after the exchange) against the default chain on C2: the same solve up to the rounding of adding the
    damping last (same steps, cost 1e-12 relative, rotations 1e-10, translations 1e-6 mm)."""
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    s0, p0 = _solve_env(pa, {}, monkeypatch)
    s1, p1 = _solve_env(pa, {"SG_XCHG_MERGE": "force"}, monkeypatch)
    assert s1["ok"] == 1 and s1["sync_timeouts"] == 0
    assert s0["num_iterations"] == s1["num_iterations"]
    assert s0["num_successful_steps"] == s1["num_successful_steps"]
    assert abs(s0["final_cost"] - s1["final_cost"]) <= 1e-12 * s0["final_cost"]
    np.testing.assert_allclose(p1.q, p0.q, rtol=0, atol=1e-10)
    np.testing.assert_allclose(p1.t, p0.t, rtol=0, atol=1e-6)


def test_rccl_communicator_on_one_rank(gpu_lib, monkeypatch):
    """The product communicator (RcclComm: ncclCommInitRank on a unique id, ncclAllReduce on the solver's stream)
    with one rank, its collectives forced (SG_COMM_FORCE=1) through the merged exchange chain (SG_XCHG_MERGE=force):
    the load's max all-reduces, the camera-block and packed-band all-reduces, each an RCCL copy on one rank.  The
    solve equals the same chain without a communicator bit for bit.  (RCCL needs one GPU per rank; the pool's
    boxes have one, so more ranks run at the driver's 8-GPU bench only.)"""
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    o = default_solver_options(max_num_iterations=6)
    s0, p0 = _solve_env(pa, {"SG_XCHG_MERGE": "force"}, monkeypatch, options=o)
    monkeypatch.setenv("SG_XCHG_MERGE", "force")
    monkeypatch.setenv("SG_COMM_FORCE", "1")
    g = ba.BundleAdjuster()
    g.comm_init(ba.BundleAdjuster.unique_id(), 1, 0)
    p1 = pa.copy()
    g.load(p1)
    s1 = g.solve(o)
    n_ar = g.info()["num_allreduces"]
    g.close()
    assert n_ar >= 7, n_ar
    assert s0 == s1
    np.testing.assert_array_equal(p0.q, p1.q)
    np.testing.assert_array_equal(p0.X, p1.X)
