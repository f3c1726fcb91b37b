"""GPU parity tests of the device HessianTracker (libslamgpu.so, sg_tracker_*) against the oracle
(oracle/oracle_track.cpp).  The device follows the oracle operation for operation (FMA contraction off,
fixed lane-tree order for the patch sums), so pyramids, patches, tracked positions, acceptance flags and
iteration counts are compared bit for bit."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import oracle  # noqa: E402
from slamgpu.tracker import HessianTracker  # noqa: E402
from slamgpu.video import ground_truth, make_frames, seed_points  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frames():
    return make_frames(2)


def _odd_image(seed=5, w=211, h=97):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)


def test_pyramid_bit_exact(gpu_lib, frames):
    for img in (frames[0], _odd_image()):
        t = HessianTracker(window=13, depth=6)
        t.MakePyramid(img, 0)
        flat, dims = oracle.make_pyramid(img, 6)
        for l, ref in enumerate(oracle.pyramid_levels(flat, dims)):
            np.testing.assert_array_equal(t.level(0, l), ref)


@pytest.mark.parametrize("W", [13, 7, 16, 1])
def test_patches_bit_exact_including_edges(gpu_lib, frames, W):
    t = HessianTracker(window=W, depth=6)
    t.MakePyramid(frames[0], 0)
    flat, dims = oracle.make_pyramid(frames[0], 6)
    levels = oracle.pyramid_levels(flat, dims)
    rng = np.random.default_rng(W)
    for l in (0, 2, 5):
        h, w = levels[l].shape
        xy = np.concatenate([rng.uniform(-2, w + 2, (200, 1)), rng.uniform(-2, h + 2, (200, 1))], 1)
        xy[:8] = [[0, 0], [0.3, 5], [5, 0.2], [w - 1, h - 1], [w - 0.01, 3], [3, h - 0.4], [6.4, 6.6], [w, h]]
        xy = xy.astype(np.float32)
        P, M, Q = t.GetPatches(0, l, xy)
        for i in range(len(xy)):
            p, m, q = oracle.get_patch(levels[l], W, float(xy[i, 0]), float(xy[i, 1]))
            np.testing.assert_array_equal(P[i], p)
            assert M[i] == np.float32(m) and Q[i] == np.float32(q)


@pytest.mark.parametrize("W", [13, 7])
def test_fb_tracking_bit_exact(gpu_lib, frames, W):
    t = HessianTracker(window=W, depth=6)
    t.MakePyramid(frames[0], 0)
    t.MakePyramid(frames[1], 1)
    pf, dims = oracle.make_pyramid(frames[0])
    pt, _ = oracle.make_pyramid(frames[1])
    pts = seed_points(600)
    rng = np.random.default_rng(1)
    levels = np.where(rng.random(len(pts)) < 0.3, 6, 3).astype(np.int32)   # uncertainty > 100 -> 6 levels
    start = pts + rng.normal(0, 0.5, pts.shape).astype(np.float32)          # projected starting guesses
    out, acc, its = t.TrackFeatureFB(0, 1, pts, start, levels)
    ro, racc, rits = oracle.track_fb(pf, pt, dims, W, pts, start, levels, nthreads=8)
    np.testing.assert_array_equal(acc.astype(np.int32), racc)
    np.testing.assert_array_equal(its, rits)
    np.testing.assert_array_equal(out, ro)
    gt = ground_truth(pts, 1)
    assert acc.mean() > 0.97
    assert np.median(np.linalg.norm(out - gt, axis=1)[acc]) < 0.15


def test_fb_rejections_and_retry_bit_exact(gpu_lib, frames):
    """Unrelated target image (most features fail, exercising the 3 -> 6 retry from the updated to_pt) and
    features at the image border (OUT_OF_BOUNDS)."""
    noise = _odd_image(seed=9, w=640, h=480)
    t = HessianTracker(window=13, depth=6)
    t.MakePyramid(frames[0], 0)
    t.MakePyramid(noise, 1)
    pf, dims = oracle.make_pyramid(frames[0])
    pn, _ = oracle.make_pyramid(noise)
    pts = np.concatenate([seed_points(300), [[0.005, 100.0], [639.999, 200.0], [3.0, 3.0], [636.5, 477.5]]]
                         ).astype(np.float32)
    out, acc, its = t.TrackFeatureFB(0, 1, pts, pts)
    ro, racc, rits = oracle.track_fb(pf, pn, dims, 13, pts, pts, nthreads=8)
    np.testing.assert_array_equal(acc.astype(np.int32), racc)
    np.testing.assert_array_equal(its, rits)
    np.testing.assert_array_equal(out, ro)
    assert acc.mean() < 0.5


def test_device_resident_runs_repeat_identically(gpu_lib, frames):
    t = HessianTracker(window=7, depth=3)
    t.MakePyramid(frames[0], 0)
    t.MakePyramid(frames[1], 1)
    pts = seed_points(2000)
    t.load_features(pts, pts)
    t.run(0, 1, repeats=3)
    o1, a1, i1 = t.results()
    t.run(0, 1, repeats=1)
    o2, a2, i2 = t.results()
    np.testing.assert_array_equal(o1, o2)
    np.testing.assert_array_equal(a1, a2)
    tm, pm = t.kernel_ms()
    assert tm > 0 and pm > 0


def test_c3_config_fb_tracking_bit_exact(gpu_lib, frames):
    """BASELINE config 3 exactly as bench.py runs it: 640x480, 2000 seeds, 3-level pyramid, 7x7 window,
    forward + backward (matcher.cpp:173-206) from the seed positions, 3 levels without the matcher's 6-level
    retry (the pyramid has 3).  The device-resident run (sg_tracker_load_features / run / results) against the
    oracle, bit for bit."""
    pts = seed_points(2000)
    t = HessianTracker(window=7, depth=3, retry_levels=0)
    t.MakePyramid(frames[0], 0)
    t.MakePyramid(frames[1], 1)
    t.load_features(pts, pts)
    t.run(0, 1, repeats=1)
    out, acc, its = t.results()
    pf, dims = oracle.make_pyramid(frames[0], 3)
    pt, _ = oracle.make_pyramid(frames[1], 3)
    ro, racc, rits = oracle.track_fb(pf, pt, dims, 7, pts, pts, np.full(len(pts), 3, np.int32),
                                     nthreads=min(16, os.cpu_count() or 1), retry_levels=0)
    np.testing.assert_array_equal(acc.astype(np.int32), racc)
    np.testing.assert_array_equal(its, rits)
    np.testing.assert_array_equal(out, ro)
    gt = ground_truth(pts, 1)
    assert acc.mean() > 0.98
    assert np.median(np.linalg.norm(out - gt, axis=1)[acc]) < 0.1
