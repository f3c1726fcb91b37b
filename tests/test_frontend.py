"""Matcher::Track (matcher.cpp:301-405): the device front end with its bookkeeping (csrc/frontend.cpp through
slamgpu.frontend.Matcher) against the sequential restatement (oracle/oracle_matcher.py) over a synthetic
sequence that exercises every branch: first-frame seeding, plain tracking frames (>= 40 matches, view not
kept), partial scene cuts (keyframes with surviving matches plus grid-filtered new corners), view expiry
after more than four keyframes, MISMATCHED features dropped, points with uncertainty < 100 starting from
their projection (3 levels) and the others from the stored match (6 levels).

CPU tests check the restatement itself against the sequence's known motion; the GPU test requires the
device run to reproduce the restatement exactly: the same matches, observations (bit-exact float
positions), keyframes, added corners and new point locations (1e-12)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import oracle_matcher as om  # noqa: E402

from slamgpu.video import SEQ_K as K, matcher_sequence as make_sequence  # noqa: E402
from slamgpu.video import sequence_mark as _mark, sequence_pose as _pose, sequence_true_t as _true_t  # noqa: E402


def run_oracle(frames):
    omap = om.OracleMap(K, [], [], [])
    mt = om.OracleMatcher()
    log = []
    for i, img in enumerate(frames):
        q, t = _pose(i)
        omap.q.append(list(q))
        omap.t.append(list(t))
        omap.frame_camera.append(0)
        omap.obs[i] = []
        omap.keyframe.append(0)
        _mark(i, omap.flags, omap.uncertainty, len(omap.X))

        def upd(i=i):   # Matcher::Track's update_frames: correct the new frame's pose, report it updated
            omap.t[i] = list(_true_t(i))
            return i % 2 == 1
        assert mt.Track(img, i, omap, upd)
        log.append(dict(mt.last_stats))
    return omap, mt, log


@pytest.fixture(scope="module")
def sequence():
    return make_sequence()


@pytest.fixture(scope="module")
def oracle_run(oracle_lib, sequence):
    return run_oracle(sequence[0])


def test_oracle_matcher_branches(oracle_run):
    omap, mt, log = oracle_run
    assert log[0]["keyframe"] == 1 and log[0]["matches"] == 0 and log[0]["added"] == log[0]["corners"] > 40
    assert log[1]["keyframe"] == 0 and log[1]["matches"] >= 40           # plain tracking frame
    cuts = [i for i, s in enumerate(log) if s["keyframe"] and s["matches"] > 0]
    assert cuts, "no keyframe with surviving matches"
    for i in cuts:    # grid filter: new corners are fewer than all corners when matches exist
        assert log[i]["added"] <= log[i]["corners"]
    assert max(s["views"] for s in log) == om.MAX_VIEWS
    assert sum(s["keyframe"] for s in log) > om.MAX_VIEWS                # view expiry exercised
    assert all(omap.keyframe[i] == log[i]["keyframe"] for i in range(len(log)))
    assert any(s["matches"] > s["matches_first"] for s in log), "update_frames re-match never added a match"


def test_oracle_matcher_tracks_follow_known_motion(oracle_run, sequence):
    """On the frames without a cut, every tracked observation of a point first seen on frame 0 sits where the
    known image shift puts it (sub-pixel tracking accuracy)."""
    omap, _, _ = oracle_run
    _, shifts = sequence
    first = {p: (x, y) for x, y, p in omap.obs[0]}
    errs = []
    for f in (1, 2):
        for x, y, p in omap.obs[f]:
            if p in first:
                ex = first[p][0] + shifts[f][0] - x
                ey = first[p][1] + shifts[f][1] - y
                errs.append(np.hypot(ex, ey))
    assert len(errs) > 80 and np.median(errs) < 0.05 and np.percentile(errs, 95) < 0.2 and max(errs) < 1.5


def test_unproject_pixel_to_plane_known_answers():
    # identity pose: the principal point unprojects onto the optical axis at the given distance
    X = om.unproject([0, 0, 0, 1], [0, 0, 0], om.pixel_to_plane(list(K), 160.0, 120.0), 2000.0)
    np.testing.assert_allclose(np.array(X[:3]) / X[3], [0, 0, 2000.0], atol=1e-9)
    assert abs(np.linalg.norm(X) - 1) < 1e-15
    # PixelToPlane inverts PlaneToPixel without distortion; Unproject then Project returns the pixel
    import oracle
    q, t = _pose(3)
    for px, py in [(10.5, 20.25), (300.0, 230.0), (160.0, 5.0)]:
        X = om.unproject(list(q), list(t), om.pixel_to_plane(list(K), px, py), 2000.0)
        uv, ok = oracle.project(q, t, K, np.array(X))
        assert ok[0] and np.allclose(uv[0], [px, py], atol=1e-9)


@pytest.mark.gpu
def test_matcher_track_matches_oracle(gpu_lib, oracle_run, sequence):
    from slamgpu.frontend import Matcher, add_frame
    from slamgpu.scene import MapArrays
    omap, omt, olog = oracle_run
    frames, _ = sequence
    z = lambda dt: np.zeros(0, dt)  # noqa: E731
    m = MapArrays(k=K.copy(), q=z(np.float64), t=z(np.float64), frame_camera=z(np.int32), frame_prev=z(np.int32),
                  X=z(np.float64), point_flags=z(np.int32), point_uncertainty=z(np.float64), obs_pt=z(np.float64),
                  obs_frame=z(np.int32), obs_point=z(np.int32), obs_disabled=z(np.int32), obs_error=z(np.float64),
                  frame_keyframe=z(np.int32))
    mt = Matcher(window=13, depth=6)
    for i, img in enumerate(frames):
        q, t = _pose(i)
        add_frame(m, 0, q, t)
        _mark(i, m.point_flags, m.point_uncertainty, m.num_points)

        def upd(i=i):
            m.t[3 * i:3 * i + 3] = _true_t(i)
            return i % 2 == 1
        assert mt.Track(img, i, 0, m, upd)
        st = mt.last_stats
        for key in ("matches_first", "matches", "keyframe", "corners", "added", "features", "views"):
            assert st[key] == olog[i][key], (i, key, st[key], olog[i][key])
        got = [(float(m.obs_pt[2 * o]), float(m.obs_pt[2 * o + 1]), int(m.obs_point[o]))
               for o in np.nonzero(m.obs_frame == i)[0]]
        assert got == omap.obs[i], "frame %d observations differ" % i
    assert m.num_points == len(omap.X)
    np.testing.assert_allclose(m.X.reshape(-1, 4), np.array(omap.X), rtol=0, atol=1e-12)
    np.testing.assert_array_equal(m.point_flags, np.array(omap.flags))
    np.testing.assert_array_equal(m.frame_keyframe, np.array(omap.keyframe))
    pts, ids = mt.features()
    assert list(ids) == sorted(omt.features) and list(pts) == [omt.features[f]["point"] for f in sorted(omt.features)]
    mt.close()


@pytest.mark.gpu
def test_failing_callback_does_not_leak_pyramid_slots(gpu_lib, sequence, monkeypatch):
    """A Track call whose callback fails (here point_state) returns the error and gives its pyramid slot back:
    with the minimum of max_images = 5 slots, many failed calls are followed by normal tracking."""
    import slamgpu.frontend as fe
    from slamgpu.scene import MapArrays
    frames, _ = sequence
    z = lambda dt: np.zeros(0, dt)  # noqa: E731
    m = MapArrays(k=K.copy(), q=z(np.float64), t=z(np.float64), frame_camera=z(np.int32), frame_prev=z(np.int32),
                  X=z(np.float64), point_flags=z(np.int32), point_uncertainty=z(np.float64), obs_pt=z(np.float64),
                  obs_frame=z(np.int32), obs_point=z(np.int32), obs_disabled=z(np.int32), obs_error=z(np.float64),
                  frame_keyframe=z(np.int32))
    mt = fe.Matcher(window=13, depth=6, max_images=5)
    q, t = _pose(0)
    fe.add_frame(m, 0, q, t)
    assert mt.Track(frames[0], 0, 0, m)       # seeds features: the first keyframe view keeps a slot
    assert m.num_points > 0

    def broken(flags):
        raise RuntimeError("point_state failed")
    monkeypatch.setattr(fe, "feature_usable", broken)
    for _ in range(8):
        with pytest.raises(RuntimeError, match="point_state failed"):
            mt.Track(frames[1], 0, 0, m)
    monkeypatch.undo()
    for i in (1, 2):
        q, t = _pose(i)
        fe.add_frame(m, 0, q, t)
        assert mt.Track(frames[i], i, 0, m)
    mt.close()
