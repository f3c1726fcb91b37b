"""Synthetic local-mapping scenes in LocalMap structure-of-arrays form.

The reference has no datasets or fixtures for this path, so benchmarks and parity tests run on
seeded synthetic scenes shaped like the robot's own data (main.cpp:474-552):

  * two pinhole cameras k = (0,0,0, 416,-416, 320,240), 640x480, alternating by frame id
    (main.cpp:474-482, 506-508: the first frame uses camera 1);
  * stereo-like pairs 150 mm apart along the camera x axis, advancing 100 mm per pair with +-3 deg
    yaw jitter (main.cpp:496, 544);
  * points uniform in the birth frame's frustum, depth U[1000, 6000] mm, stored as unit-norm
    homogeneous locations (localmap.cpp:35), uncertainty 1.0, flags clear (slam-usable);
  * each point observed in a contiguous run of frames starting at its birth frame, run length
    U{run_min..run_max}, cut where it leaves the image; N(0, 0.5 px) pixel noise, 1 % outliers U(+-20 px);
  * initial perturbation of the free frames (0.5 deg rotation, 10 mm translation) and of the points
    (5 % depth along the birth ray).  The two oldest frames keep their true pose (gauge).

Configs (BASELINE.json): C1 = 10 KF / 500 pts (seed 1), C2 = 50 KF / 20k pts / ~150k obs (seed 2),
C5 = 200 KF / 200k pts / ~2M obs (seed 5).  run_min sets the observation count per landmark without widening
the co-visibility band (run_max bounds it).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from .capi import SgMap, ptr

WIDTH, HEIGHT = 640, 480
K_ROBOT = np.array([0.0, 0.0, 0.0, 416.0, -416.0, 320.0, 240.0])

CONFIGS = {
    "C1": dict(num_frames=10, num_points=500, seed=1, run_max=14),
    "C2": dict(num_frames=50, num_points=20000, seed=2, run_max=14, run_min=4),
    "C5": dict(num_frames=200, num_points=200000, seed=5, run_max=18, run_min=6),
}


def quat_from_matrix(R: np.ndarray) -> np.ndarray:
    """Rotation matrix -> Eigen quaternion coeffs [x, y, z, w] (w >= 0)."""
    m = R
    tr = m[0, 0] + m[1, 1] + m[2, 2]
    if tr > 0:
        s = np.sqrt(tr + 1.0) * 2
        w, x, y, z = 0.25 * s, (m[2, 1] - m[1, 2]) / s, (m[0, 2] - m[2, 0]) / s, (m[1, 0] - m[0, 1]) / s
    elif m[0, 0] > m[1, 1] and m[0, 0] > m[2, 2]:
        s = np.sqrt(1.0 + m[0, 0] - m[1, 1] - m[2, 2]) * 2
        w, x, y, z = (m[2, 1] - m[1, 2]) / s, 0.25 * s, (m[0, 1] + m[1, 0]) / s, (m[0, 2] + m[2, 0]) / s
    elif m[1, 1] > m[2, 2]:
        s = np.sqrt(1.0 + m[1, 1] - m[0, 0] - m[2, 2]) * 2
        w, x, y, z = (m[0, 2] - m[2, 0]) / s, (m[0, 1] + m[1, 0]) / s, 0.25 * s, (m[1, 2] + m[2, 1]) / s
    else:
        s = np.sqrt(1.0 + m[2, 2] - m[0, 0] - m[1, 1]) * 2
        w, x, y, z = (m[1, 0] - m[0, 1]) / s, (m[0, 2] + m[2, 0]) / s, (m[1, 2] + m[2, 1]) / s, 0.25 * s
    q = np.array([x, y, z, w])
    return q if w >= 0 else -q


def quat_to_matrix(q: np.ndarray) -> np.ndarray:
    x, y, z, w = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def rot_y(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def axis_angle(v):
    th = np.linalg.norm(v)
    if th == 0:
        return np.eye(3)
    k = v / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def project_np(R, t, k, Xw):
    """Vectorised project.h for Euclidean world points (rows) with per-row R (n,3,3), t (n,3)."""
    p = np.einsum("nij,nj->ni", R, Xw - t)
    ok = p[:, 2] > 1e-9
    z = np.where(ok, p[:, 2], 1.0)
    xp, yp = p[:, 0] / z, p[:, 1] / z
    r2 = xp * xp + yp * yp
    d = 1 + r2 * (k[0] + r2 * (k[1] + r2 * k[2]))
    return np.stack([k[3] * d * xp + k[5], k[4] * d * yp + k[6]], 1), ok


@dataclass
class MapArrays:
    """LocalMap (localmap.h:284-320) as numpy arrays; .struct() gives the sg_map view."""
    k: np.ndarray              # [ncam*7]
    q: np.ndarray              # [F*4] Eigen [x,y,z,w]
    t: np.ndarray              # [F*3]
    frame_camera: np.ndarray   # [F] int32
    frame_prev: np.ndarray     # [F] int32
    X: np.ndarray              # [P*4]
    point_flags: np.ndarray    # [P] int32
    point_uncertainty: np.ndarray  # [P]
    obs_pt: np.ndarray         # [M*2]
    obs_frame: np.ndarray      # [M] int32
    obs_point: np.ndarray      # [M] int32
    obs_disabled: np.ndarray   # [M] int32
    obs_error: np.ndarray      # [M*2]
    frame_keyframe: np.ndarray = None   # [F] int32 Frame::is_keyframe_ (set by Matcher::Track)
    # ground truth (not part of the map)
    q_true: np.ndarray = None
    t_true: np.ndarray = None
    X_true: np.ndarray = None

    @property
    def num_frames(self):
        return len(self.frame_camera)

    @property
    def num_points(self):
        return len(self.point_flags)

    @property
    def num_obs(self):
        return len(self.obs_frame)

    def copy(self) -> "MapArrays":
        return MapArrays(**{f: (getattr(self, f).copy() if getattr(self, f) is not None else None)
                            for f in self.__dataclass_fields__})

    def struct(self) -> SgMap:
        m = SgMap()
        m.num_cameras = len(self.k) // 7
        m.k = ptr(self.k, C.c_double)
        m.num_frames = self.num_frames
        m.q, m.t = ptr(self.q, C.c_double), ptr(self.t, C.c_double)
        m.frame_camera, m.frame_prev = ptr(self.frame_camera, C.c_int32), ptr(self.frame_prev, C.c_int32)
        m.num_points = self.num_points
        m.X = ptr(self.X, C.c_double)
        m.point_flags = ptr(self.point_flags, C.c_int32)
        m.point_uncertainty = ptr(self.point_uncertainty, C.c_double)
        m.num_obs = self.num_obs
        m.obs_pt = ptr(self.obs_pt, C.c_double)
        m.obs_frame, m.obs_point = ptr(self.obs_frame, C.c_int32), ptr(self.obs_point, C.c_int32)
        m.obs_disabled = ptr(self.obs_disabled, C.c_int32)
        m.obs_error = ptr(self.obs_error, C.c_double)
        return m


def make_scene(num_frames: int, num_points: int, seed: int, run_max: int = 14, run_min: int = 2, noise: float = 0.5,
               outlier_frac: float = 0.01, outlier_px: float = 20.0, rot_noise_deg: float = 0.5,
               trans_noise: float = 10.0, depth_noise: float = 0.05, num_const: int = 2,
               perturb: bool = True) -> MapArrays:
    rng = np.random.default_rng(seed)
    F, P = num_frames, num_points
    k = np.concatenate([K_ROBOT, K_ROBOT])
    # --- trajectory: frame f is side (f % 2) of stereo pair f // 2
    R_true = np.zeros((F, 3, 3))
    t_true = np.zeros((F, 3))
    yaw = np.deg2rad(rng.uniform(-3.0, 3.0, size=(F + 1) // 2))
    for f in range(F):
        j, side = divmod(f, 2)
        R = rot_y(yaw[j])                       # world -> camera
        c = np.array([0.0, 0.0, 100.0 * j])
        if side:
            c = c + R.T @ np.array([150.0, 0.0, 0.0])
        R_true[f], t_true[f] = R, c
    frame_camera = ((np.arange(F) + 1) % 2).astype(np.int32)
    frame_prev = (np.arange(F) - 1).astype(np.int32)

    # --- points: born in a frame's frustum, observed over a contiguous run of frames
    birth = rng.integers(0, F - 1, size=P)
    u = rng.uniform(16.0, WIDTH - 16.0, size=P)
    v = rng.uniform(16.0, HEIGHT - 16.0, size=P)
    depth = rng.uniform(1000.0, 6000.0, size=P)
    xp = (u - K_ROBOT[5]) / K_ROBOT[3]
    yp = (v - K_ROBOT[6]) / K_ROBOT[4]
    pc = np.stack([xp * depth, yp * depth, depth], 1)
    Xw = np.einsum("nji,nj->ni", R_true[birth], pc) + t_true[birth]
    run = rng.integers(run_min, run_max + 1, size=P)
    obs_list = []   # (frame, point, u, v)
    nobs = np.zeros(P, dtype=np.int64)
    alive = np.ones(P, dtype=bool)
    for ell in range(run_max):
        fr = birth + ell
        act = alive & (ell < run) & (fr < F)
        idx = np.nonzero(act)[0]
        if idx.size == 0:
            break
        f_idx = fr[idx]
        uv, ok = project_np(R_true[f_idx], t_true[f_idx], K_ROBOT, Xw[idx])
        inside = ok & (uv[:, 0] >= 0) & (uv[:, 0] < WIDTH) & (uv[:, 1] >= 0) & (uv[:, 1] < HEIGHT)
        alive[idx[~inside]] = False
        idx, f_idx, uv = idx[inside], f_idx[inside], uv[inside]
        obs_list.append((f_idx, idx, uv))
        nobs[idx] += 1
    keep = nobs >= 2   # points with one observation stay NO_OBSERVATIONS in the reference: drop them
    remap = -np.ones(P, dtype=np.int64)
    remap[keep] = np.arange(keep.sum())
    Xw = Xw[keep]
    birth = birth[keep]
    P = int(keep.sum())
    frames, points, uvs = [], [], []
    for f_idx, idx, uv in obs_list:
        m = keep[idx]
        frames.append(f_idx[m]); points.append(remap[idx[m]]); uvs.append(uv[m])
    obs_frame = np.concatenate(frames).astype(np.int32)
    obs_point = np.concatenate(points).astype(np.int32)
    uv = np.concatenate(uvs)
    M = len(obs_frame)
    uv = uv + rng.normal(0.0, noise, size=uv.shape)
    outl = rng.random(M) < outlier_frac
    uv[outl] += rng.uniform(-outlier_px, outlier_px, size=(int(outl.sum()), 2))
    # order observations by frame, then point (Frame::observations() order)
    order = np.lexsort((obs_point, obs_frame))
    obs_frame, obs_point, uv = obs_frame[order], obs_point[order], uv[order]

    # --- initial estimate
    q0 = np.zeros((F, 4))
    t0 = t_true.copy()
    q_true = np.stack([quat_from_matrix(R) for R in R_true])
    Xw0 = Xw.copy()
    for f in range(F):
        R = R_true[f]
        if perturb and f >= num_const:
            R = axis_angle(rng.normal(size=3) / np.sqrt(3) * np.deg2rad(rot_noise_deg)) @ R
            t0[f] = t_true[f] + rng.normal(0.0, trans_noise, size=3)
        q0[f] = quat_from_matrix(R)
    if perturb:
        c = t_true[birth]
        Xw0 = c + (Xw - c) * (1.0 + rng.normal(0.0, depth_noise, size=(P, 1)))
    Xh = np.concatenate([Xw0, np.ones((P, 1))], 1)
    Xh /= np.linalg.norm(Xh, axis=1, keepdims=True)
    Xh_true = np.concatenate([Xw, np.ones((P, 1))], 1)
    Xh_true /= np.linalg.norm(Xh_true, axis=1, keepdims=True)
    return MapArrays(
        k=k, q=q0.reshape(-1).copy(), t=t0.reshape(-1).copy(), frame_camera=frame_camera,
        frame_prev=frame_prev, X=Xh.reshape(-1).copy(), point_flags=np.zeros(P, dtype=np.int32),
        point_uncertainty=np.ones(P), obs_pt=uv.reshape(-1).copy(), obs_frame=obs_frame,
        obs_point=obs_point, obs_disabled=np.zeros(M, dtype=np.int32), obs_error=np.zeros(2 * M),
        q_true=q_true.reshape(-1), t_true=t_true.reshape(-1), X_true=Xh_true.reshape(-1))


def make_config(name: str, **overrides) -> MapArrays:
    cfg = dict(CONFIGS[name])
    cfg.update(overrides)
    return make_scene(**cfg)
