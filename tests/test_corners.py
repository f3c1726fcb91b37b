"""New-keyframe corner seeding: Matcher::Track's cvtColor(RGB2GRAY) +
goodFeaturesToTrack(grey, 120, 0.01, 20) + AddNewFeatures' grid filter (matcher.cpp:123-169, 214).

OpenCV is not available here and the reference holds no fixture for this path, so parity with OpenCV is
unpinned; the oracle (oracle_track.cpp, restating OpenCV 2.4's corner.cpp / featureselect.cpp) is pinned by
known-answer tests (isolated squares: the corners are found at the square corners, strongest first,
minimum distance respected, the grid filter drops exactly the corners near matches).  The device path
(corners.hip) is compared with the oracle bit-exactly: same corners, same order, same added subset.
"""
import numpy as np
import pytest

from slamgpu.video import make_frames


def _squares(w=640, h=480, side=30, step=80, seed=0):
    """Bright squares on a dark background (BGR, grey replicated)."""
    rng = np.random.default_rng(seed)
    img = np.full((h, w), 20, np.uint8)
    tops = []
    for y0 in range(40, h - side - 40, step):
        for x0 in range(40, w - side - 40, step):
            img[y0:y0 + side, x0:x0 + side] = 200 + rng.integers(0, 40)
            tops.append((x0, y0))
    return np.repeat(img[:, :, None], 3, axis=2), tops, side


def test_oracle_corners_known_answer(oracle_lib):
    img, tops, side = _squares()
    corners, added = oracle_lib.seed_features(img, None, max_corners=120)
    assert len(corners) == 120 and np.array_equal(corners, added)
    truth = np.array([(x + dx, y + dy) for x, y in tops for dx in (0, side - 1) for dy in (0, side - 1)], float)
    d = np.sqrt(((corners[:, None, :] - truth[None, :, :]) ** 2).sum(-1)).min(1)
    assert d.max() <= 1.5, d.max()          # every corner sits on a square corner
    # minimum distance and strongest-first order
    pd = np.sqrt(((corners[:, None, :] - corners[None, :, :]) ** 2).sum(-1)) + np.eye(len(corners)) * 1e9
    assert pd.min() >= 20.0
    eig = oracle_lib.min_eigen(img)
    resp = eig[corners[:, 1].astype(int), corners[:, 0].astype(int)]
    assert np.all(np.diff(resp) <= 0)


def test_oracle_grid_filter(oracle_lib):
    img = make_frames(1)[0]
    corners, added = oracle_lib.seed_features(img)
    matches = corners[::3] + 0.25
    c2, a2 = oracle_lib.seed_features(img, matches)
    np.testing.assert_array_equal(c2, corners)
    h, w = img.shape[:2]
    cell = lambda p: (int(np.float32(p[0]) / np.float32(w) * np.float32(30) + np.float32(1)),
                      int(np.float32(p[1]) / np.float32(h) * np.float32(30) + np.float32(1)))
    blocked = set()
    for m in matches:
        gx, gy = cell(m)
        blocked |= {(gx + a, gy + b) for a in (-1, 0, 1) for b in (-1, 0, 1)}
    expect = np.array([c for c in corners if cell(c) not in blocked], np.float32).reshape(-1, 2)
    np.testing.assert_array_equal(a2, expect)
    assert 0 < len(a2) < len(corners)
    with pytest.raises(ValueError):
        oracle_lib.seed_features(img, np.array([[w + 5.0, 10.0]], np.float32))


def test_oracle_corners_parameters(oracle_lib):
    img = make_frames(1)[0]
    c_all, _ = oracle_lib.seed_features(img, max_corners=1000, min_distance=5.0)
    c_few, _ = oracle_lib.seed_features(img, max_corners=50, min_distance=5.0)
    np.testing.assert_array_equal(c_few, c_all[:50])   # greedy prefix property
    flat = np.full((480, 640, 3), 77, np.uint8)
    c, a = oracle_lib.seed_features(flat)
    assert len(c) == 0 and len(a) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["video", "squares", "dense"])
def test_seed_features_gpu_matches_oracle(gpu_lib, oracle_lib, case):
    from slamgpu.tracker import HessianTracker
    if case == "squares":
        img = _squares()[0]
        kw = {}
    else:
        img = make_frames(2)[1]
        kw = dict(max_corners=1000, min_distance=5.0) if case == "dense" else {}
    t = HessianTracker(window=13, depth=3)
    t.MakePyramid(img, 0)
    co, ao = oracle_lib.seed_features(img, None, **kw)
    cg, ag = t.SeedFeatures(0, None, **kw)
    np.testing.assert_array_equal(cg, co)
    np.testing.assert_array_equal(ag, ao)
    matches = co[::4] + 0.5
    co2, ao2 = oracle_lib.seed_features(img, matches, **kw)
    cg2, ag2 = t.SeedFeatures(0, matches, **kw)
    np.testing.assert_array_equal(cg2, co2)
    np.testing.assert_array_equal(ag2, ao2)
    t.close()
