"""Synthetic KLT video (BASELINE config 3): 640x480 u8 grey replicated to 3 channels,
texture = Gaussian-blurred (sigma 2) uniform noise (seed 3); frame t = texture warped by translation
t*(0.7, -0.4) px plus a 0.2 deg * t rotation about the image centre (known ground truth); feature seeds on
a jittered grid >= 10 px from the border."""
from __future__ import annotations

import numpy as np
from scipy import ndimage


def _texture(w, h, seed, margin=64):
    rng = np.random.default_rng(seed)
    t = rng.uniform(0.0, 255.0, size=(h + 2 * margin, w + 2 * margin))
    return ndimage.gaussian_filter(t, 2.0), margin


def frame_motion(t: float, w: int = 640, h: int = 480):
    """Ground-truth map from frame-0 pixel coordinates to frame-t coordinates: x_t = R (x_0 - c) + c + d."""
    ang = np.deg2rad(0.2 * t)
    c, s = np.cos(ang), np.sin(ang)
    R = np.array([[c, -s], [s, c]])
    d = np.array([0.7 * t, -0.4 * t])
    ctr = np.array([(w - 1) / 2.0, (h - 1) / 2.0])
    return R, d, ctr


def make_frames(n_frames: int = 2, w: int = 640, h: int = 480, seed: int = 3):
    tex, m = _texture(w, h, seed)
    frames = []
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float64)
    for t in range(n_frames):
        R, d, ctr = frame_motion(t, w, h)
        # inverse warp: frame_t(x) = tex(R^T (x - c - d) + c)
        px = xs - ctr[0] - d[0]
        py = ys - ctr[1] - d[1]
        sx = R[0, 0] * px + R[1, 0] * py + ctr[0]
        sy = R[0, 1] * px + R[1, 1] * py + ctr[1]
        img = ndimage.map_coordinates(tex, [sy + m, sx + m], order=1, mode="nearest")
        g = np.clip(np.rint(img), 0, 255).astype(np.uint8)
        frames.append(np.repeat(g[:, :, None], 3, axis=2))
    return frames


def seed_points(n: int = 2000, w: int = 640, h: int = 480, border: float = 10.0, seed: int = 3):
    """n seeds on a jittered grid at least `border` px inside the image."""
    rng = np.random.default_rng(seed + 100)
    aspect = (w - 2 * border) / (h - 2 * border)
    ny = int(np.ceil(np.sqrt(n / aspect)))
    nx = int(np.ceil(n / ny))
    gx = np.linspace(border + 2, w - border - 2, nx)
    gy = np.linspace(border + 2, h - border - 2, ny)
    X, Y = np.meshgrid(gx, gy)
    pts = np.stack([X.ravel(), Y.ravel()], 1)[:n]
    pts += rng.uniform(-1.0, 1.0, pts.shape)
    return np.clip(pts, border, [w - border, h - border]).astype(np.float32)


def ground_truth(pts: np.ndarray, t: float, w: int = 640, h: int = 480):
    R, d, ctr = frame_motion(t, w, h)
    return ((pts - ctr) @ R.T + ctr + d).astype(np.float32)


# ---------------------------------------------------------------------------------------------------------
# Matcher::Track sequence (matcher.cpp:301-405): tests/test_frontend.py checks the device front end on it
# against the sequential restatement, and bench.py times it per frame.  320 x 240, every branch of Track:
# first-frame seeding, plain tracking frames, partial scene cuts (keyframes with surviving matches and
# grid-filtered new corners), view expiry, MISMATCHED points dropped, projected (3-level) and stored
# (6-level) starting points.

SEQ_W, SEQ_H = 320, 240
SEQ_K = np.array([0.0, 0.0, 0.0, 416.0, -416.0, 160.0, 120.0])   # main.cpp:474-482 intrinsics, centred
# (texture seed of the left part, fraction of the width covered by that fresh texture)
SEQ_SCHEDULE = [(None, 0.0), (None, 0.0), (None, 0.0), (11, 0.8), (11, 0.8), (12, 0.85), (13, 0.9), (13, 0.9),
                (14, 0.9), (15, 0.9), (None, 0.0)]
_MISMATCHED = 3   # TrackedPoint flag bit (localmap.h)


def _seq_texture(seed, margin=48):
    rng = np.random.default_rng(seed)
    t = rng.uniform(0.0, 255.0, size=(SEQ_H + 2 * margin, SEQ_W + 2 * margin))
    return ndimage.gaussian_filter(t, 2.0), margin


def _seq_warp(tex, m, dx, dy):
    ys, xs = np.mgrid[0:SEQ_H, 0:SEQ_W].astype(np.float64)
    return ndimage.map_coordinates(tex, [ys - dy + m, xs - dx + m], order=1, mode="nearest")


def matcher_sequence():
    """(frames as (h, w, 3) u8 BGR, per-frame image shift of the base texture)."""
    base, m = _seq_texture(3)
    frames, shifts = [], []
    for i, (seed, frac) in enumerate(SEQ_SCHEDULE):
        dx, dy = 0.7 * i, -0.4 * i
        img = _seq_warp(base, m, dx, dy)
        if seed is not None:
            other, m2 = _seq_texture(seed)
            cut = int(frac * SEQ_W)
            img[:, :cut] = _seq_warp(other, m2, 0.5 * i, 0.3 * i)[:, :cut]
        g = np.clip(np.rint(img), 0, 255).astype(np.uint8)
        frames.append(np.repeat(g[:, :, None], 3, axis=2))
        shifts.append((dx, dy))
    return frames, shifts


def sequence_true_t(i):
    """Camera translation that moves a point 2000 mm ahead by the base texture's image shift (0.7, -0.4) px per
    frame (fx = 416, fy = -416)."""
    return np.array([-0.7 * i * 2000 / 416, -0.4 * i * 2000 / 416, 0.0])


def sequence_pose(i):
    """Initial pose guess: identity rotation; odd frames from 3 on start 100 mm off (about 20 px), which
    update_frames then corrects (the role SolveFramePose would have)."""
    t = sequence_true_t(i)
    if i >= 3 and i % 2 == 1:
        t = t + np.array([100.0, 0.0, 0.0])
    return np.array([0.0, 0.0, 0.0, 1.0]), t


def sequence_mark(step, flags, unc, npts):
    """Between frames: mark some points MISMATCHED and give some an uncertainty below 100 (Clean's role)."""
    if step == 5 and npts > 10:
        flags[3] |= 1 << _MISMATCHED
        flags[7] |= 1 << _MISMATCHED
    if step in (2, 6):
        for p in range(0, npts, 3):
            unc[p] = 3.0
        for p in range(1, npts, 6):
            unc[p] = 100.0
