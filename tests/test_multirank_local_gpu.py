"""The landmark-sharded device chain on ONE GPU.

Two solver handles on device 0, each driven by its own host thread, exchange through the in-process
communicator group (sg_comm_group: stream sync, host barrier, rank-ordered device sum) instead of RCCL.  The
solver's compute path is the multi-rank one: the Cholesky envelope is the union of the shards' envelopes
(load-time max all-reduce), only rank 0 assembles the camera-only terms, S and its rhs travel packed
(k_S_pack), and every rank takes the replicated accept/reject decision (k_decide).  Parity: against the
one-rank solve of the whole problem (which differs from the sharded one only in summation order).

Also here, since they need the device: a validation failure on one rank fails every rank (no hang), a point
observed 3000 times (the Schur segment that does not stage its rows in LDS), and a load that fails followed
by a reload of the previous problem.
"""
import threading

import numpy as np
import pytest

from slamgpu import ba
from slamgpu.capi import ProblemArrays, SlamGpuError, default_solver_options
from slamgpu.scene import make_config, make_scene

pytestmark = pytest.mark.gpu


def _sharded(pa, nranks, options=None, shards=None, timeout=240):
    """Solve the nranks landmark shards of pa through one in-process group; returns per-rank
    (summary, shard problem after the solve, info) or the exception each rank raised."""
    group = ba.LocalCommGroup(nranks)
    shards = shards or [ba.shard_problem(pa, r, nranks) for r in range(nranks)]
    out = [None] * nranks

    def work(r):
        try:
            g = ba.BundleAdjuster()
            g.comm_init_local(group, r)
            g.load(shards[r])
            info = g.info()
            s = g.solve(options)
            out[r] = (s, shards[r], info)
            g.close()
        except Exception as e:   # noqa: BLE001 - reported per rank
            out[r] = e

    th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    assert not any(t.is_alive() for t in th), "a rank did not finish"
    group.close()
    return out


def _merge_points(pa, results):
    """Solved points of every shard, in pa's point order (matched by point_map_index)."""
    X = np.full_like(pa.X, np.nan)
    where = {int(m): i for i, m in enumerate(pa.point_map_index)}
    for s, sh, _ in results:
        for j, m in enumerate(sh.point_map_index):
            i = where[int(m)]
            X[4 * i:4 * i + 4] = sh.X[4 * j:4 * j + 4]
    assert not np.isnan(X).any()
    return X


def _check_against_one_rank(pa, results, options, cost_rtol, q_atol, t_atol, X_atol):
    for r in results:
        assert not isinstance(r, Exception), r
    s0, sh0, i0 = results[0]
    # replicated decision and factorisation: every rank holds the same frames and the same summary
    for s, sh, info in results[1:]:
        assert s == s0
        np.testing.assert_array_equal(sh.q, sh0.q)
        np.testing.assert_array_equal(sh.t, sh0.t)
    for s, sh, info in results:
        assert info["nranks"] == len(results) and info["n"] == i0["n"]
        assert info["band_tiles"] == i0["band_tiles"]   # the envelope union: every rank factors the same band
    one = pa.copy()
    g = ba.BundleAdjuster()
    g.load(one)
    s1 = g.solve(options)
    i1 = g.info()
    assert i1["band_tiles"] == i0["band_tiles"] and i1["cholesky_path"] == i0["cholesky_path"]
    assert s0["num_iterations"] == s1["num_iterations"]
    assert s0["num_successful_steps"] == s1["num_successful_steps"]
    assert abs(s0["initial_cost"] - s1["initial_cost"]) <= 1e-12 * s1["initial_cost"]
    assert abs(s0["final_cost"] - s1["final_cost"]) <= cost_rtol * s1["final_cost"]
    np.testing.assert_allclose(sh0.q, one.q, rtol=0, atol=q_atol)
    np.testing.assert_allclose(sh0.t, one.t, rtol=0, atol=t_atol)
    np.testing.assert_allclose(_merge_points(pa, results), one.X, rtol=0, atol=X_atol)
    return s0, s1


def test_two_shards_c2_first_iterations_match_one_rank(gpu_lib):
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    o = default_solver_options(max_num_iterations=5)
    res = _sharded(pa, 2, o)
    _check_against_one_rank(pa, res, o, 1e-12, 1e-10, 1e-6, 1e-10)
    # Schur work balance of sg_problem_shard's split (first observing frame, balanced by observations)
    pairs = [info["num_pairs"] for _, _, info in res]
    obs = [sh.num_obs for _, sh, _ in res]
    assert max(pairs) / (sum(pairs) / 2) <= 1.25, pairs
    assert max(obs) / (sum(obs) / 2) <= 1.1, obs


def test_two_shards_c2_converged_solve_matches_one_rank(gpu_lib):
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    o = default_solver_options()
    res = _sharded(pa, 2, o)
    for r in res:
        assert not isinstance(r, Exception), r
    s0, sh0, _ = res[0]
    one = pa.copy()
    g = ba.BundleAdjuster()
    g.load(one)
    s1 = g.solve(o)
    assert s0["ok"] == s1["ok"] == 1
    assert s0["termination"] == "FUNCTION_TOLERANCE"
    assert abs(s0["num_iterations"] - s1["num_iterations"]) <= 2
    assert abs(s0["final_cost"] - s1["final_cost"]) <= 1e-7 * s1["final_cost"]
    np.testing.assert_allclose(sh0.t, one.t, rtol=0, atol=1e-3)
    np.testing.assert_allclose(sh0.q, one.q, rtol=0, atol=1e-7)


def test_four_shards_wide_scene_match_one_rank(gpu_lib):
    """Points over > 24 free frames (global-atomic wide path), constant points, a skipped frame, disabled
    observations, four shards."""
    m = make_scene(num_frames=40, num_points=2000, seed=21, run_max=40)
    rng = np.random.default_rng(0)
    m.obs_disabled[rng.random(m.num_obs) < 0.05] = 1
    m.obs_disabled[m.obs_frame == 30] = 1
    pa = ba.problem_from_map_frames(m, 38, 40, 2.0)
    o = default_solver_options(max_num_iterations=3)
    res = _sharded(pa, 4, o)
    _check_against_one_rank(pa, res, o, 1e-11, 1e-9, 1e-5, 1e-9)


def test_two_shards_c5_first_iterations_match_one_rank(gpu_lib):
    m = make_config("C5")
    pa = ba.problem_from_map_frames(m, 198, 200, 2.0)
    o = default_solver_options(max_num_iterations=2)
    res = _sharded(pa, 2, o)
    _check_against_one_rank(pa, res, o, 1e-12, 1e-10, 1e-6, 1e-10)


@pytest.mark.parametrize("nranks", [4, 8])
def test_many_shards_c5_first_iterations_match_one_rank(gpu_lib, nranks):
    """BASELINE config 5 split into nranks landmark shards (8: the 8-GPU split config 5 names), each driven by
    its own host thread and handle on one GPU through the in-process group: the sharded device chain (envelope
    union, rank-0 assembly, packed band exchange, replicated factorisation and decision) against the one-rank
    solve of the whole problem, two LM iterations."""
    m = make_config("C5")
    pa = ba.problem_from_map_frames(m, 198, 200, 2.0)
    o = default_solver_options(max_num_iterations=2)
    res = _sharded(pa, nranks, o, timeout=600)
    s0, _ = _check_against_one_rank(pa, res, o, 1e-12, 1e-10, 1e-6, 1e-10)
    assert s0["sync_timeouts"] == 0
    obs = [sh.num_obs for _, sh, _ in res]
    assert max(obs) / (sum(obs) / nranks) <= 1.1, obs


def test_eight_shards_c2_match_one_rank(gpu_lib):
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    o = default_solver_options(max_num_iterations=5)
    res = _sharded(pa, 8, o, timeout=300)
    s0, _ = _check_against_one_rank(pa, res, o, 1e-12, 1e-10, 1e-6, 1e-10)
    assert s0["sync_timeouts"] == 0


def test_invalid_shard_fails_every_rank(gpu_lib):
    """A rank whose problem fails validation must not leave its peers blocked in the load-time all-reduce."""
    m = make_config("C1")
    pa = ba.problem_from_map_frames(m, 8, 10, 2.0)
    shards = [ba.shard_problem(pa, r, 2) for r in range(2)]
    shards[1].obs_point[0] = 10 ** 6   # out of range
    res = _sharded(pa, 2, shards=shards, timeout=120)
    assert all(isinstance(r, SlamGpuError) for r in res), res
    assert "out of range" in str(res[1]) or "obs_point" in str(res[1])
    assert "another landmark shard" in str(res[0])


def _heavy_point_problem(nobs_heavy=3000):
    """C1-sized problem plus one free point observed nobs_heavy times (spread over the free frames, each
    observation its own pixel noise): a whole-map solve's long-tracked point."""
    m = make_config("C1")
    pa = ba.problem_from_map_frames(m, 8, 10, 2.0)
    rng = np.random.default_rng(3)
    i = int(np.nonzero(pa.point_free)[0][0])
    src = np.nonzero(pa.obs_point == i)[0]
    pick = rng.choice(src, size=nobs_heavy, replace=True)
    obs_pt = np.concatenate([pa.obs_pt, pa.obs_pt.reshape(-1, 2)[pick].reshape(-1) +
                             rng.normal(0, 0.5, size=2 * nobs_heavy)])
    return ProblemArrays(pa.k, pa.q, pa.t, pa.frame_camera, pa.frame_rot_free, pa.frame_trans_free, pa.X,
                         pa.point_free, obs_pt, np.concatenate([pa.obs_frame, pa.obs_frame[pick]]),
                         np.concatenate([pa.obs_point, pa.obs_point[pick]]), pa.dist_frame, pa.dist_prev,
                         pa.range, pa.cameras_free, pa.frame_map_index, pa.point_map_index)


def test_heavily_observed_point_matches_oracle(gpu_lib, oracle_lib):
    pa = _heavy_point_problem()
    o = default_solver_options(max_num_iterations=2)
    pg, po = pa.copy(), pa.copy()
    g = ba.BundleAdjuster()
    g.load(pg)
    sg = g.solve(o)
    so = oracle_lib.solve(po, o)
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]
    np.testing.assert_allclose(pg.t, po.t, rtol=0, atol=1e-6)
    np.testing.assert_allclose(pg.X, po.X, rtol=0, atol=1e-9)


def test_failed_load_then_reload(gpu_lib):
    """A load rejected by validation (a point with 65536 observations) leaves the handle's previous problem
    intact: reloading that problem solves exactly like a fresh handle."""
    m = make_config("C1")
    pa = ba.problem_from_map_frames(m, 8, 10, 2.0)
    bad = _heavy_point_problem(65536)
    g = ba.BundleAdjuster()
    g.load(pa.copy())
    with pytest.raises(SlamGpuError, match="65536"):
        g.load(bad)
    # the device chain is deterministic (k_schur: MFMA accumulators in point order; fixed-order partial
    # reductions), so the reloaded handle and a fresh one agree bit for bit
    o = default_solver_options(max_num_iterations=3)
    p1 = pa.copy()
    g.load(p1)
    s1 = g.solve(o)
    p2 = pa.copy()
    f = ba.BundleAdjuster()
    f.load(p2)
    s2 = f.solve(o)
    assert s1["num_iterations"] == s2["num_iterations"] == 4
    assert s1 == s2
    np.testing.assert_array_equal(p1.X, p2.X)
    np.testing.assert_array_equal(p1.q, p2.q)


def _sharded_counts(pa, nranks, first, more):
    """Begin + `first` iterations, then `more` iterations on every shard; per rank (all-reduces issued during
    the `more` iterations, summary, shard after download)."""
    group = ba.LocalCommGroup(nranks)
    shards = [ba.shard_problem(pa, r, nranks) for r in range(nranks)]
    out = [None] * nranks

    def work(r):
        try:
            g = ba.BundleAdjuster()
            g.comm_init_local(group, r)
            g.load(shards[r])
            g.begin(default_solver_options(max_num_iterations=first + more))
            g.iterate(first)
            g.sync()
            c0 = g.info()["num_allreduces"]
            g.iterate(more)
            g.sync()
            c1 = g.info()["num_allreduces"]
            s = g.summary()
            g.download()
            out[r] = (c1 - c0, s, shards[r])
            g.close()
        except Exception as e:   # noqa: BLE001 - reported per rank
            out[r] = e

    th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not any(t.is_alive() for t in th), "a rank did not finish"
    group.close()
    for r in out:
        assert not isinstance(r, Exception), r
    return out


@pytest.mark.parametrize("merge", ["1", "0"], ids=["merged", "three-exchange"])
def test_exchanges_per_iteration(gpu_lib, monkeypatch, merge):
    """After a solve's first iteration (which sums the camera blocks, then S, then the step scalars: three
    all-reduces) the shards exchange twice per LM iteration: the band of S with the camera gradient, diagonal and
    cost scalars in its tail, then the step scalars (SG_XCHG_MERGE=0 keeps three).  Both chains give
    the one-rank solve of C2 to rounding: 4 shards, 6 iterations."""
    monkeypatch.setenv("SG_XCHG_MERGE", merge)
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    out = _sharded_counts(pa, 4, 1, 5)
    for n_ar, s, sh in out:
        assert n_ar == 5 * (2 if merge == "1" else 3), n_ar
        np.testing.assert_array_equal(sh.q, out[0][2].q)   # replicated decision: every rank the same poses
        assert s == out[0][1]
    monkeypatch.delenv("SG_XCHG_MERGE")
    (_, s1, one), = _sharded_counts(pa, 1, 1, 5)   # the one-rank handle, the same begin / iterate sequence
    s0 = out[0][1]
    assert s0["num_successful_steps"] == s1["num_successful_steps"]
    assert abs(s0["final_cost"] - s1["final_cost"]) <= 1e-12 * s1["final_cost"]
    np.testing.assert_allclose(out[0][2].q, one.q, rtol=0, atol=1e-10)
    np.testing.assert_allclose(out[0][2].t, one.t, rtol=0, atol=1e-6)
