"""Python mirror of the reference's Matcher (matcher.h:13-31) over sg_frontend_* (csrc/frontend.cpp), and the
LocalMap growth it needs on the SoA map (slamgpu.scene.MapArrays).

`Matcher.Track(img, frame, camera, map, update_frames)` is Matcher::Track (matcher.cpp:301-405): the
bookkeeping runs in the library's host C++, every image operation on the device.  The map stays the
caller's: the library reads and grows it through the sg_map_callbacks implemented here.  New observations
are inserted at the end of their frame's group (Frame::AddObservation, localmap.h:138-143); new points are
appended (LocalMap::AddPoint, localmap.cpp:103-109).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .capi import (ADD_OBS_CB, ADD_POINT_CB, FRAME_POSE_CB, POINT_STATE_CB, SET_KEYFRAME_CB, UPDATE_FRAMES_CB,
                   SgDeviceOptions, SgFrontendStats, SgMapCallbacks, check, load_library)
from .scene import MapArrays
from .tracker import default_tracker_options

NO_BASELINE, NO_OBSERVATIONS, MISMATCHED, BAD_LOCATION = 1, 2, 3, 0


def feature_usable(flags: int) -> bool:
    """TrackedPoint::feature_usable (localmap.h:249)."""
    return not (flags & (1 << MISMATCHED)) and not (flags & (1 << BAD_LOCATION))


# ---------------------------------------------------------------------------------------------------------
# LocalMap growth on MapArrays

def add_frame(m: MapArrays, camera: int, q=(0.0, 0.0, 0.0, 1.0), t=(0.0, 0.0, 0.0)) -> int:
    """LocalMap::AddFrame (localmap.cpp:92-98): the new frame's previous() is the last frame."""
    f = m.num_frames
    m.q = np.concatenate([m.q, np.asarray(q, np.float64)])
    m.t = np.concatenate([m.t, np.asarray(t, np.float64)])
    m.frame_camera = np.concatenate([m.frame_camera, np.int32([camera])])
    m.frame_prev = np.concatenate([m.frame_prev, np.int32([f - 1 if f else -1])])
    if getattr(m, "frame_keyframe", None) is not None:
        m.frame_keyframe = np.concatenate([m.frame_keyframe, np.int32([0])])
    return f


def add_points(m: MapArrays, X: np.ndarray) -> np.ndarray:
    """LocalMap::AddPoint for each row of X[n, 4]: flags NO_OBSERVATIONS | NO_BASELINE, uncertainty 1e8."""
    X = np.asarray(X, np.float64).reshape(-1, 4)
    first = m.num_points
    m.X = np.concatenate([m.X, X.reshape(-1)])
    m.point_flags = np.concatenate([m.point_flags,
                                    np.full(len(X), (1 << NO_OBSERVATIONS) | (1 << NO_BASELINE), np.int32)])
    m.point_uncertainty = np.concatenate([m.point_uncertainty, np.full(len(X), 1e8)])
    return np.arange(first, first + len(X), dtype=np.int32)


def add_observations(m: MapArrays, frame: int, xy: np.ndarray, points: np.ndarray):
    """Frame::AddObservation for each (xy[i], points[i]) in order: appended to the frame's group."""
    xy = np.asarray(xy, np.float64).reshape(-1, 2)
    n = len(xy)
    if n == 0:
        return
    if len(m.obs_frame) and np.any(np.diff(m.obs_frame) < 0):
        raise ValueError("observations are not grouped by frame")
    pos = int(np.searchsorted(m.obs_frame, frame, side="right"))
    m.obs_pt = np.insert(m.obs_pt, 2 * pos, xy.reshape(-1))
    m.obs_frame = np.insert(m.obs_frame, pos, np.full(n, frame, np.int32))
    m.obs_point = np.insert(m.obs_point, pos, np.asarray(points, np.int32))
    m.obs_disabled = np.insert(m.obs_disabled, pos, np.zeros(n, np.int32))
    m.obs_error = np.insert(m.obs_error, 2 * pos, np.zeros(2 * n))


def commit_frame(m: MapArrays, frame: int):
    """Frame::Commit (localmap.cpp:85-89): each observed point re-checks its flags (TrackedPoint::CheckFlags,
    localmap.cpp:41-83) over its observations in frame order."""
    for p in np.unique(m.obs_point[m.obs_frame == frame]):
        fl = int(m.point_flags[p])
        sel = np.nonzero((m.obs_point == p) & (m.obs_disabled == 0))[0]
        sel = sel[np.argsort(m.obs_frame[sel], kind="stable")]
        if fl & (1 << NO_OBSERVATIONS) and len(sel) >= 2:
            fl &= ~(1 << NO_OBSERVATIONS)
        if fl & (1 << NO_BASELINE) and len(sel) >= 2:
            base = m.t[3 * m.obs_frame[sel[0]]:3 * m.obs_frame[sel[0]] + 3]
            for o in sel[1:]:
                pos = m.t[3 * m.obs_frame[o]:3 * m.obs_frame[o] + 3]
                if np.linalg.norm(pos - base) >= 50:      # minimum baseline distance (localmap.cpp:70)
                    fl &= ~(1 << NO_BASELINE)
                    break
        m.point_flags[p] = fl


# ---------------------------------------------------------------------------------------------------------

class Matcher:
    """matcher.h's Matcher: Track() per frame; the live features and keyframe views live in the library."""

    def __init__(self, device: int = 0, window: int = 13, depth: int = 6, max_images: int = 8, **kw):
        self.lib = load_library()
        self.opt = default_tracker_options(window=window, depth=depth, max_images=max_images, **kw)
        self.h = C.c_void_p()
        dev = SgDeviceOptions(device=device, precision=0, rank=0, nranks=1)
        check(self.lib.sg_frontend_create(C.byref(self.h), C.byref(self.opt), C.byref(dev)), "sg_frontend_create")
        self.last_stats = None

    def close(self):
        if self.h:
            self.lib.sg_frontend_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def features(self):
        """Live features: (point index, TrackedPoint id) in set order."""
        n = C.c_int32(0)
        check(self.lib.sg_frontend_features(self.h, None, None, C.byref(n)), "sg_frontend_features")
        pts, ids = np.zeros(n.value, np.int32), np.zeros(n.value, np.int32)
        cap = C.c_int32(n.value)
        check(self.lib.sg_frontend_features(self.h, pts.ctypes.data_as(C.POINTER(C.c_int32)),
                                            ids.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(cap)),
              "sg_frontend_features")
        return pts, ids

    def Track(self, img: np.ndarray, frame: int, camera: int, m: MapArrays, update_frames=None) -> bool:
        """Matcher::Track(img, frame, camera, map, update_frames).  img: (h, w, 3) uint8, cv::Mat BGR order."""
        img = np.ascontiguousarray(img, dtype=np.uint8)
        h, w = img.shape[:2]
        if getattr(m, "frame_keyframe", None) is None:
            m.frame_keyframe = np.zeros(m.num_frames, np.int32)
        pend_X, pend_obs = [], []
        err = []

        def flush():
            if pend_X:
                add_points(m, np.array(pend_X))
                pend_X.clear()
            by_frame = {}
            for f, x, y, p in pend_obs:
                by_frame.setdefault(f, []).append((x, y, p))
            for f, lst in by_frame.items():
                add_observations(m, f, [(x, y) for x, y, _ in lst], [p for _, _, p in lst])
            pend_obs.clear()

        def guard(fn):
            def wrapped(*a):
                try:
                    return fn(*a)
                except BaseException as e:     # surfaces after the C call returns
                    err.append(e)
                    return 1
            return wrapped

        @guard
        def frame_pose(_u, f, q, t, k):
            c = int(m.frame_camera[f])
            for i in range(4):
                q[i] = float(m.q[4 * f + i])
            for i in range(3):
                t[i] = float(m.t[3 * f + i])
            for i in range(7):
                k[i] = float(m.k[7 * c + i])
            return 0

        @guard
        def point_state(_u, p, X, unc, usable):
            for i in range(4):
                X[i] = float(m.X[4 * p + i])
            unc[0] = float(m.point_uncertainty[p])
            usable[0] = 1 if feature_usable(int(m.point_flags[p])) else 0
            return 0

        @guard
        def add_point(_u, pid, X, out):
            pend_X.append([X[i] for i in range(4)])
            out[0] = m.num_points + len(pend_X) - 1
            return 0

        @guard
        def add_obs(_u, f, x, y, p):
            pend_obs.append((f, x, y, p))
            return 0

        @guard
        def set_keyframe(_u, f):
            m.frame_keyframe[f] = 1
            return 0

        @guard
        def upd(_u, out):
            flush()       # the reference's observations are already in the frame when update_frames runs
            out[0] = 1 if update_frames() else 0
            return 0

        cbs = SgMapCallbacks(None, FRAME_POSE_CB(frame_pose), POINT_STATE_CB(point_state), ADD_POINT_CB(add_point),
                             ADD_OBS_CB(add_obs), SET_KEYFRAME_CB(set_keyframe),
                             UPDATE_FRAMES_CB(upd) if update_frames is not None else UPDATE_FRAMES_CB())
        res = C.c_int32(0)
        st = SgFrontendStats()
        rc = self.lib.sg_frontend_track(self.h, img.ctypes.data_as(C.POINTER(C.c_uint8)), w, h, img.strides[0],
                                        frame, camera, C.byref(cbs), C.byref(res), C.byref(st))
        if err:
            raise err[0]
        check(rc, "sg_frontend_track")
        flush()
        self.last_stats = st.as_dict()
        return bool(res.value)
