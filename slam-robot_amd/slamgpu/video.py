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
