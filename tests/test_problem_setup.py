"""CPU tests of the host side of the boundary: Slam::SetupProblem rules (slam.cpp:257-443) as implemented
in libslamgpu.so (sg_problem_from_map_*), checked against the oracle's independent restatement, plus the
landmark-shard partition used by the multi-GPU path.  No GPU needed (these are host-only entry points)."""
import numpy as np
import pytest

from slamgpu import ba
from slamgpu.capi import BAD_FEATURE, NO_BASELINE, NO_OBSERVATIONS
from slamgpu.scene import make_config, make_scene


def _same(pa, po):
    assert (pa is None) == (po is None)
    if pa is None:
        return
    for f in pa.FIELDS:
        np.testing.assert_array_equal(getattr(pa, f), getattr(po, f), err_msg=f)
    assert pa.range == po.range and pa.cameras_free == po.cameras_free


def _edge_map(seed=11):
    m = make_scene(num_frames=14, num_points=600, seed=seed, run_max=8)
    rng = np.random.default_rng(seed)
    m.obs_disabled[rng.random(m.num_obs) < 0.1] = 1
    m.point_flags[rng.random(m.num_points) < 0.03] |= 1 << NO_BASELINE
    m.point_flags[rng.random(m.num_points) < 0.03] |= 1 << BAD_FEATURE
    m.point_flags[rng.random(m.num_points) < 0.02] |= 1 << NO_OBSERVATIONS
    m.point_uncertainty[rng.random(m.num_points) < 0.2] = 500.0     # "not quite sure": solved anyway
    # frame 9 presented but unusable -> skipped; frame 10's FrameDistance gets a free translation block
    m.obs_disabled[m.obs_frame == 9] = 1
    return m


@pytest.mark.parametrize("solve,present", [(8, 10), (2, 5), (10, 20), (1, 14), (14, 14), (5, 6), (0, 4)])
def test_solve_frames_setup_matches_oracle(oracle_lib, solve, present):
    for m in (make_config("C1"), _edge_map(), _edge_map(12)):
        pa = ba.problem_from_map_frames(m, solve, present, 2.0)
        po = oracle_lib.problem_from_map_frames(m, solve, present, 2.0)
        _same(pa, po)


def test_skipped_previous_frame_gets_free_translation_block(oracle_lib):
    m = _edge_map()
    pa = ba.problem_from_map_frames(m, 5, 8, 2.0)   # frames 9..13 free, 6..8 const: 9 is skipped
    fm = list(pa.frame_map_index)
    # frame 9 has no usable observation -> not a rotation block; it is frame 10's previous frame
    assert 9 in fm
    i9 = fm.index(9)
    assert pa.frame_rot_free[i9] == 0 and pa.frame_trans_free[i9] == 1
    i10 = fm.index(10)
    assert any(a == i10 and b == i9 for a, b in zip(pa.dist_frame, pa.dist_prev))
    _same(pa, oracle_lib.problem_from_map_frames(m, 5, 8, 2.0))


def test_point_constness_rule(oracle_lib):
    m = _edge_map()
    pa = ba.problem_from_map_frames(m, 3, 9, 2.0)
    free_frames = {pa.frame_map_index[i] for i in range(pa.num_frames) if pa.frame_rot_free[i]}
    for i in range(pa.num_points):
        mp = pa.point_map_index[i]
        obs = (m.obs_point == mp) & (m.obs_disabled == 0)
        seen_by_free = any(f in free_frames for f in m.obs_frame[obs])
        expect_const = m.point_uncertainty[mp] <= 100 and not seen_by_free
        assert pa.point_free[i] == (not expect_const)


def test_too_few_frames_aborts(oracle_lib):
    m = make_config("C1")
    assert ba.problem_from_map_frames(m, 1, 1, 2.0) is None
    assert oracle_lib.problem_from_map_frames(m, 1, 1, 2.0) is None
    m.obs_disabled[:] = 1
    assert ba.problem_from_map_frames(m, 8, 10, 2.0) is None


@pytest.mark.parametrize("cams", [False, True])
def test_solve_all_frames_setup_matches_oracle(oracle_lib, cams):
    for m in (make_config("C1"), _edge_map()):
        _same(ba.problem_from_map_all(m, 2.0, cams), oracle_lib.problem_from_map_all(m, 2.0, cams))


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_landmark_shards_partition_the_problem(nranks):
    m = make_config("C1")
    pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    shards = [ba.shard_problem(pa, r, nranks) for r in range(nranks)]
    pts = np.concatenate([s.point_map_index for s in shards])
    assert sorted(pts.tolist()) == sorted(pa.point_map_index.tolist())
    assert sum(s.num_obs for s in shards) == pa.num_obs
    for s in shards:
        np.testing.assert_array_equal(s.q, pa.q)
        np.testing.assert_array_equal(s.t, pa.t)
        np.testing.assert_array_equal(s.dist_frame, pa.dist_frame)
        # each observation travels with its point
        for o in range(0, s.num_obs, 17):
            mp = s.point_map_index[s.obs_point[o]]
            src = np.nonzero((pa.point_map_index[pa.obs_point] == mp) &
                             (pa.obs_frame == s.obs_frame[o]))[0]
            assert len(src) >= 1
            assert np.allclose(pa.obs_pt.reshape(-1, 2)[src[0]], s.obs_pt.reshape(-1, 2)[o])
    if nranks > 1:
        counts = np.array([s.num_obs for s in shards])
        assert counts.max() <= 1.5 * pa.num_obs / nranks + 50


def _permuted(m, order):
    m = m.copy()
    for f in ("obs_frame", "obs_point", "obs_disabled"):
        setattr(m, f, np.ascontiguousarray(getattr(m, f)[order]))
    for f in ("obs_pt", "obs_error"):
        v = getattr(m, f)
        if v is not None:
            setattr(m, f, np.ascontiguousarray(v.reshape(-1, 2)[order].reshape(-1)))
    return m


@pytest.mark.parametrize("solve,present", [(2, 5), (10, 20), (14, 14)])
def test_setup_with_observations_out_of_frame_order(oracle_lib, solve, present):
    """A LocalMap's observations come ordered by frame, and the setup then walks only the presented frames'
    range; any other order takes the full walk.  Both give the oracle's problem (observations in map order)."""
    base = _edge_map()
    assert np.all(np.diff(base.obs_frame) >= 0)   # the fast path's precondition holds for the scene maps
    rng = np.random.default_rng(5)
    last_first = np.r_[1:base.num_obs, 0]          # one observation of frame 0 moved to the end
    for order in (rng.permutation(base.num_obs), last_first):
        m = _permuted(base, order)
        _same(ba.problem_from_map_frames(m, solve, present, 2.0),
              oracle_lib.problem_from_map_frames(m, solve, present, 2.0))
