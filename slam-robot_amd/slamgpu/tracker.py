"""Device HessianTracker (hessian.h) and the matcher's forward/backward step (matcher.cpp:173-206, 247-251)
behind the C-ABI (include/slamgpu.h, sg_tracker_*).

Method names follow the reference: MakePyramid builds a view's pyramid (into a device slot), GetPatch /
GetPatches sample patches, TrackFeatureFB is matcher.cpp's TrackFeature (forward + backward + 0.3 px check)
including FindMatches' retry with 6 levels.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .capi import SgDeviceOptions, SgTrackerOptions, check, load_library


def _dev(device=0):
    return SgDeviceOptions(device=device, precision=0, rank=0, nranks=1)

_fp = C.POINTER(C.c_float)
_ip = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)
_dp = C.POINTER(C.c_double)


def default_tracker_options(**kw) -> SgTrackerOptions:
    lib = load_library()
    o = SgTrackerOptions()
    lib.sg_tracker_options_default(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


class HessianTracker:
    def __init__(self, window: int = 13, depth: int = 6, device: int = 0, max_images: int = 8, **kw):
        self.lib = load_library()
        self.opt = default_tracker_options(window=window, depth=depth, max_images=max_images, **kw)
        self.h = C.c_void_p()
        dev = _dev(device)
        check(self.lib.sg_tracker_create(C.byref(self.h), C.byref(self.opt), C.byref(dev)), "sg_tracker_create")

    def close(self):
        if self.h:
            self.lib.sg_tracker_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def window(self) -> int:
        return self.opt.window

    def MakePyramid(self, img: np.ndarray, slot: int = 0):
        """hessian.h:95-126.  img: (h, w, 3) uint8 in cv::Mat (BGR) memory order."""
        img = np.ascontiguousarray(img, dtype=np.uint8)
        h, w = img.shape[:2]
        check(self.lib.sg_tracker_set_image(self.h, slot, img.ctypes.data_as(_u8p), w, h, img.strides[0]),
              "sg_tracker_set_image")
        return slot

    def level(self, slot: int, level: int) -> np.ndarray:
        w, h = C.c_int32(), C.c_int32()
        check(self.lib.sg_tracker_get_level(self.h, slot, level, None, C.byref(w), C.byref(h)), "get_level")
        out = np.zeros((h.value, w.value), np.float32)
        check(self.lib.sg_tracker_get_level(self.h, slot, level, out.ctypes.data_as(_fp), C.byref(w), C.byref(h)),
              "get_level")
        return out

    def GetPatches(self, slot: int, level: int, xy: np.ndarray):
        """GetPatch (hessian.h:54-93) at many points: (patches[n, W, W], mean[n], sumsq[n])."""
        xy = np.ascontiguousarray(xy, dtype=np.float32).reshape(-1, 2)
        n, W = xy.shape[0], self.window
        out = np.zeros((n, W, W), np.float32)
        mean = np.zeros(n, np.float32)
        sumsq = np.zeros(n, np.float32)
        check(self.lib.sg_tracker_get_patches(self.h, slot, level, n, xy.ctypes.data_as(_fp), out.ctypes.data_as(_fp),
                                              mean.ctypes.data_as(_fp), sumsq.ctypes.data_as(_fp)), "get_patches")
        return out, mean, sumsq

    def TrackFeatureFB(self, from_slot: int, to_slot: int, from_xy, to_xy=None, levels=None):
        """matcher.cpp TrackFeature for many features.  Returns (to_xy, accepted[bool], iterations)."""
        from_xy = np.ascontiguousarray(from_xy, dtype=np.float32).reshape(-1, 2)
        n = from_xy.shape[0]
        out = (from_xy.copy() if to_xy is None else np.ascontiguousarray(to_xy, dtype=np.float32).reshape(-1, 2).copy())
        lv = np.full(n, 3, np.int32) if levels is None else np.ascontiguousarray(levels, dtype=np.int32)
        acc = np.zeros(n, np.int32)
        its = np.zeros(n, np.int32)
        check(self.lib.sg_tracker_track(self.h, from_slot, to_slot, n, from_xy.ctypes.data_as(_fp),
                                        out.ctypes.data_as(_fp), lv.ctypes.data_as(_ip), acc.ctypes.data_as(_ip),
                                        its.ctypes.data_as(_ip)), "sg_tracker_track")
        return out, acc.astype(bool), its

    # device-resident throughput path (bench)
    def load_features(self, from_xy, to_xy, levels=None):
        from_xy = np.ascontiguousarray(from_xy, dtype=np.float32).reshape(-1, 2)
        to_xy = np.ascontiguousarray(to_xy, dtype=np.float32).reshape(-1, 2)
        n = from_xy.shape[0]
        lv = np.full(n, 3, np.int32) if levels is None else np.ascontiguousarray(levels, dtype=np.int32)
        self._n = n
        check(self.lib.sg_tracker_load_features(self.h, n, from_xy.ctypes.data_as(_fp), to_xy.ctypes.data_as(_fp),
                                                lv.ctypes.data_as(_ip)), "load_features")

    def run(self, from_slot: int, to_slot: int, repeats: int = 1):
        check(self.lib.sg_tracker_run(self.h, from_slot, to_slot, repeats), "sg_tracker_run")

    def results(self):
        n = self._n
        out = np.zeros((n, 2), np.float32)
        acc = np.zeros(n, np.int32)
        its = np.zeros(n, np.int32)
        check(self.lib.sg_tracker_results(self.h, out.ctypes.data_as(_fp), acc.ctypes.data_as(_ip),
                                          its.ctypes.data_as(_ip)), "sg_tracker_results")
        return out, acc.astype(bool), its

    def kernel_ms(self):
        t, p = C.c_double(), C.c_double()
        check(self.lib.sg_tracker_kernel_ms(self.h, C.byref(t), C.byref(p)), "kernel_ms")
        return t.value, p.value

    def TrackFeature(self, from_slot: int, to_slot: int, from_xy, to_xy=None, levels=None):
        """One-directional TrackFeature of this tracker's mode (hessian.h:243-264 / klt.h:403-424 /
        brute.h:129-164) for many features: GetPatches(from_slot, from_xy), then tracking in to_slot from to_xy.
        Returns (to_xy, status (0 OK, 2 OUT_OF_BOUNDS), iterations); failed features keep their guess."""
        from_xy = np.ascontiguousarray(from_xy, dtype=np.float32).reshape(-1, 2)
        n = from_xy.shape[0]
        out = (from_xy.copy() if to_xy is None else np.ascontiguousarray(to_xy, dtype=np.float32).reshape(-1, 2).copy())
        lv = None if levels is None else np.ascontiguousarray(levels, dtype=np.int32)
        st = np.zeros(n, np.int32)
        its = np.zeros(n, np.int32)
        check(self.lib.sg_tracker_track_feature(self.h, from_slot, to_slot, n, from_xy.ctypes.data_as(_fp),
                                                out.ctypes.data_as(_fp), None if lv is None else lv.ctypes.data_as(_ip),
                                                st.ctypes.data_as(_ip), its.ctypes.data_as(_ip)),
              "sg_tracker_track_feature")
        return out, st, its

    def SeedFeatures(self, slot: int, match_xy=None, max_corners: int = 120, quality: float = 0.01,
                     min_distance: float = 20.0):
        """Matcher::Track's new-keyframe seeding on the image of `slot` (matcher.cpp:123-169, AddNewFeatures):
        goodFeaturesToTrack(grey, 120, 0.01, 20) then the 30 x 30 grid filter against the current matches.
        Returns (corners[n, 2], added[m, 2])."""
        mxy = np.ascontiguousarray(np.zeros((0, 2)) if match_xy is None else match_xy, dtype=np.float32).reshape(-1, 2)
        corners = np.zeros((max_corners, 2), np.float32)
        added = np.zeros((max_corners, 2), np.float32)
        nc, na = C.c_int32(), C.c_int32()
        check(self.lib.sg_tracker_seed_features(self.h, slot, mxy.ctypes.data_as(_fp) if len(mxy) else None, len(mxy),
                                                max_corners, quality, min_distance, corners.ctypes.data_as(_fp),
                                                C.byref(nc), added.ctypes.data_as(_fp), C.byref(na)),
              "sg_tracker_seed_features")
        return corners[:nc.value].copy(), added[:na.value].copy()


class KLTTracker(HessianTracker):
    """klt.h's KLTTracker on the device (sg_tracker_options.mode = SG_TRACKER_KLT): MakePyramid and
    TrackFeature with klt.h's pyramid, masked SSD and forward-difference Newton step."""

    def __init__(self, window: int = 13, depth: int = 6, device: int = 0, max_images: int = 8, **kw):
        super().__init__(window=window, depth=depth, device=device, max_images=max_images, mode=1, **kw)


class BruteTracker(HessianTracker):
    """brute.h's BruteTracker on the device (sg_tracker_options.mode = SG_TRACKER_BRUTE): exhaustive
    float-stepped SearchBest grids, one candidate per thread."""

    def __init__(self, window: int = 13, depth: int = 6, device: int = 0, max_images: int = 8, **kw):
        super().__init__(window=window, depth=depth, device=device, max_images=max_images, mode=2, **kw)
