"""ctypes mirror of include/slamgpu.h and the loader for libslamgpu.so.

The structures here are the C-ABI boundary (include/slamgpu.h); nothing in this module computes.
`load_library()` fails loudly when the HIP library has not been built: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC_DIR = os.path.join(os.path.dirname(PKG_DIR), "csrc")
# SG_LIB_PATH: an alternative in-tree build of the same library (A/B of kernel variants: tools/)
LIB_PATH = os.environ.get("SG_LIB_PATH") or os.path.join(CSRC_DIR, "libslamgpu.so")

SG_OK = 0
TERMINATION = {0: "NO_CONVERGENCE", 1: "FUNCTION_TOLERANCE", 2: "GRADIENT_TOLERANCE",
               3: "PARAMETER_TOLERANCE", 4: "NUMERICAL_FAILURE", 5: "DID_NOT_RUN",
               6: "DEVICE_TIMEOUT"}

# TrackedPoint::Flags bit positions (localmap.h:184-190)
BAD_LOCATION, NO_BASELINE, NO_OBSERVATIONS, MISMATCHED, BAD_FEATURE = range(5)

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)


class SgMap(C.Structure):
    _fields_ = [
        ("num_cameras", C.c_int32), ("k", _dp),
        ("num_frames", C.c_int32), ("q", _dp), ("t", _dp), ("frame_camera", _ip), ("frame_prev", _ip),
        ("num_points", C.c_int32), ("X", _dp), ("point_flags", _ip), ("point_uncertainty", _dp),
        ("num_obs", C.c_int32), ("obs_pt", _dp), ("obs_frame", _ip), ("obs_point", _ip),
        ("obs_disabled", _ip), ("obs_error", _dp),
    ]


class SgProblem(C.Structure):
    _fields_ = [
        ("num_cameras", C.c_int32), ("k", _dp), ("cameras_free", C.c_int32),
        ("num_frames", C.c_int32), ("q", _dp), ("t", _dp), ("frame_camera", _ip),
        ("frame_rot_free", _u8p), ("frame_trans_free", _u8p), ("frame_map_index", _ip),
        ("num_points", C.c_int32), ("X", _dp), ("point_free", _u8p), ("point_map_index", _ip),
        ("num_obs", C.c_int32), ("obs_pt", _dp), ("obs_frame", _ip), ("obs_point", _ip),
        ("num_dist", C.c_int32), ("dist_frame", _ip), ("dist_prev", _ip),
        ("range", C.c_double), ("dist_target", C.c_double), ("dist_range", C.c_double),
        ("stab_range", C.c_double), ("owner_", C.c_void_p),
    ]


class SgSolverOptions(C.Structure):
    _fields_ = [
        ("max_num_iterations", C.c_int32), ("function_tolerance", C.c_double),
        ("gradient_tolerance", C.c_double), ("parameter_tolerance", C.c_double),
        ("min_relative_decrease", C.c_double), ("initial_trust_region_radius", C.c_double),
        ("max_trust_region_radius", C.c_double), ("min_trust_region_radius", C.c_double),
        ("min_lm_diagonal", C.c_double), ("max_lm_diagonal", C.c_double),
        ("max_num_consecutive_invalid_steps", C.c_int32), ("jacobi_scaling", C.c_int32),
        ("disable_termination", C.c_int32), ("always_linearize", C.c_int32),
    ]


class SgSolverSummary(C.Structure):
    _fields_ = [
        ("num_iterations", C.c_int32), ("num_successful_steps", C.c_int32),
        ("num_unsuccessful_steps", C.c_int32), ("num_invalid_steps", C.c_int32),
        ("termination_type", C.c_int32), ("ok", C.c_int32),
        ("initial_cost", C.c_double), ("final_cost", C.c_double), ("fixed_cost", C.c_double),
        ("trust_region_radius", C.c_double), ("num_lm_iterations", C.c_int32), ("sync_timeouts", C.c_int32),
    ]

    def as_dict(self):
        d = {name: getattr(self, name) for name, _ in self._fields_}
        d["termination"] = TERMINATION.get(self.termination_type, "?")
        return d


class SgBaInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("num_frames", "num_points", "num_obs", "num_blocks", "n", "band_tiles",
                                         "cholesky_path", "num_pairs", "rank", "nranks", "cholesky_split",
                                         "num_allreduces", "lin_waves", "cholesky_separator")]
    CHOLESKY_PATHS = {0: "tiled band (k_chol_tiles)", 1: "LDS window (k_cholesky_window)",
                      2: "global memory (k_cholesky_global, LDS-staged panel rows)",
                      3: "global memory (k_cholesky_global, unstaged)",
                      4: "bordered band (k_chol_tiles on the frames, k_chol_border for the intrinsics)"}

    def as_dict(self):
        d = {n: getattr(self, n) for n, _ in self._fields_}
        d["cholesky"] = self.CHOLESKY_PATHS.get(self.cholesky_path, "?")
        return d


class SgDeviceOptions(C.Structure):
    _fields_ = [("device", C.c_int32), ("precision", C.c_int32), ("rank", C.c_int32),
                ("nranks", C.c_int32)]


def default_solver_options(**kw) -> SgSolverOptions:
    """ceres::Solver::Options of Slam::Run (slam.cpp:486-499) with Ceres 1.8 defaults."""
    o = SgSolverOptions(
        max_num_iterations=1000, function_tolerance=1e-7, gradient_tolerance=1e-10,
        parameter_tolerance=1e-8, min_relative_decrease=1e-3, initial_trust_region_radius=1e4,
        max_trust_region_radius=1e16, min_trust_region_radius=1e-32, min_lm_diagonal=1e-6,
        max_lm_diagonal=1e32, max_num_consecutive_invalid_steps=5, jacobi_scaling=1,
        disable_termination=0, always_linearize=0)
    for key, val in kw.items():
        setattr(o, key, val)
    return o


def ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype)) if a is not None and a.size else C.POINTER(ctype)()


class ProblemArrays:
    """Caller-owned numpy storage for an sg_problem (arrays stay alive with this object)."""

    FIELDS = ("k", "q", "t", "frame_camera", "frame_rot_free", "frame_trans_free", "frame_map_index",
              "X", "point_free", "point_map_index", "obs_pt", "obs_frame", "obs_point", "dist_frame",
              "dist_prev")

    def __init__(self, k, q, t, frame_camera, frame_rot_free, frame_trans_free, X, point_free, obs_pt,
                 obs_frame, obs_point, dist_frame, dist_prev, range_=2.0, cameras_free=0,
                 frame_map_index=None, point_map_index=None, dist_target=150.0, dist_range=15.0,
                 stab_range=5.0):
        f64 = lambda a: np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
        i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32).reshape(-1)
        u8 = lambda a: np.ascontiguousarray(a, dtype=np.uint8).reshape(-1)
        self.k, self.q, self.t, self.X, self.obs_pt = f64(k), f64(q), f64(t), f64(X), f64(obs_pt)
        self.frame_camera, self.obs_frame, self.obs_point = i32(frame_camera), i32(obs_frame), i32(obs_point)
        self.dist_frame, self.dist_prev = i32(dist_frame), i32(dist_prev)
        self.frame_rot_free, self.frame_trans_free, self.point_free = (
            u8(frame_rot_free), u8(frame_trans_free), u8(point_free))
        nf, npnt = len(self.frame_camera), len(self.point_free)
        self.frame_map_index = i32(frame_map_index if frame_map_index is not None else np.arange(nf))
        self.point_map_index = i32(point_map_index if point_map_index is not None else np.arange(npnt))
        self.range, self.cameras_free = float(range_), int(cameras_free)
        self.dist_target, self.dist_range, self.stab_range = dist_target, dist_range, stab_range

    @property
    def num_frames(self):
        return len(self.frame_camera)

    @property
    def num_points(self):
        return len(self.point_free)

    @property
    def num_obs(self):
        return len(self.obs_frame)

    def copy(self) -> "ProblemArrays":
        return ProblemArrays(self.k.copy(), self.q.copy(), self.t.copy(), self.frame_camera.copy(),
                             self.frame_rot_free.copy(), self.frame_trans_free.copy(), self.X.copy(),
                             self.point_free.copy(), self.obs_pt.copy(), self.obs_frame.copy(),
                             self.obs_point.copy(), self.dist_frame.copy(), self.dist_prev.copy(),
                             self.range, self.cameras_free, self.frame_map_index.copy(),
                             self.point_map_index.copy(), self.dist_target, self.dist_range,
                             self.stab_range)

    def struct(self) -> SgProblem:
        p = SgProblem()
        p.num_cameras = len(self.k) // 7
        p.k = ptr(self.k, C.c_double)
        p.cameras_free = self.cameras_free
        p.num_frames = self.num_frames
        p.q, p.t = ptr(self.q, C.c_double), ptr(self.t, C.c_double)
        p.frame_camera = ptr(self.frame_camera, C.c_int32)
        p.frame_rot_free = ptr(self.frame_rot_free, C.c_uint8)
        p.frame_trans_free = ptr(self.frame_trans_free, C.c_uint8)
        p.frame_map_index = ptr(self.frame_map_index, C.c_int32)
        p.num_points = self.num_points
        p.X = ptr(self.X, C.c_double)
        p.point_free = ptr(self.point_free, C.c_uint8)
        p.point_map_index = ptr(self.point_map_index, C.c_int32)
        p.num_obs = self.num_obs
        p.obs_pt = ptr(self.obs_pt, C.c_double)
        p.obs_frame, p.obs_point = ptr(self.obs_frame, C.c_int32), ptr(self.obs_point, C.c_int32)
        p.num_dist = len(self.dist_frame)
        p.dist_frame, p.dist_prev = ptr(self.dist_frame, C.c_int32), ptr(self.dist_prev, C.c_int32)
        p.range, p.dist_target, p.dist_range, p.stab_range = (
            self.range, self.dist_target, self.dist_range, self.stab_range)
        p.owner_ = None
        return p

    @staticmethod
    def from_struct(p: SgProblem) -> "ProblemArrays":
        """Copy a (library- or oracle-owned) sg_problem into numpy storage."""
        def arr(pp, n, dt):
            if n == 0:
                return np.zeros(0, dtype=dt)
            return np.ctypeslib.as_array(pp, shape=(n,)).astype(dt).copy()
        nf, npnt, nm, nd, nc = p.num_frames, p.num_points, p.num_obs, p.num_dist, p.num_cameras
        return ProblemArrays(
            arr(p.k, 7 * nc, np.float64), arr(p.q, 4 * nf, np.float64), arr(p.t, 3 * nf, np.float64),
            arr(p.frame_camera, nf, np.int32), arr(p.frame_rot_free, nf, np.uint8),
            arr(p.frame_trans_free, nf, np.uint8), arr(p.X, 4 * npnt, np.float64),
            arr(p.point_free, npnt, np.uint8), arr(p.obs_pt, 2 * nm, np.float64),
            arr(p.obs_frame, nm, np.int32), arr(p.obs_point, nm, np.int32),
            arr(p.dist_frame, nd, np.int32), arr(p.dist_prev, nd, np.int32), p.range, p.cameras_free,
            arr(p.frame_map_index, nf, np.int32), arr(p.point_map_index, npnt, np.int32),
            p.dist_target, p.dist_range, p.stab_range)


_LIB = None

class SgTrackerOptions(C.Structure):
    _fields_ = [("window", C.c_int32), ("depth", C.c_int32), ("max_iterations", C.c_int32),
                ("threshold", C.c_float), ("fb_max", C.c_float), ("retry_levels", C.c_int32),
                ("max_images", C.c_int32), ("mode", C.c_int32), ("reserved", C.c_int32 * 4)]


_fp = C.POINTER(C.c_float)
_u8p = C.POINTER(C.c_uint8)

# sg_map_callbacks (slamgpu.h): the LocalMap accessors Matcher::Track uses.
FRAME_POSE_CB = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, _dp, _dp, _dp)
POINT_STATE_CB = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, _dp, _dp, C.POINTER(C.c_int32))
ADD_POINT_CB = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, _dp, C.POINTER(C.c_int32))
ADD_OBS_CB = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, C.c_double, C.c_double, C.c_int32)
SET_KEYFRAME_CB = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32)
UPDATE_FRAMES_CB = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.POINTER(C.c_int32))


class SgMapCallbacks(C.Structure):
    _fields_ = [("user", C.c_void_p), ("frame_pose", FRAME_POSE_CB), ("point_state", POINT_STATE_CB),
                ("add_point", ADD_POINT_CB), ("add_observation", ADD_OBS_CB), ("set_keyframe", SET_KEYFRAME_CB),
                ("update_frames", UPDATE_FRAMES_CB)]


class SgFrontendStats(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("matches_first", "matches", "keyframe", "corners", "added", "features",
                                         "views", "track_batches")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


# sg_allreduce_fn: int (*)(double* buf, long long n, int32_t op, void* user)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_longlong, C.c_int32, C.c_void_p)

SYMBOLS = {
    "sg_version": (C.c_char_p, []),
    "sg_last_error": (C.c_char_p, []),
    "sg_solver_options_default": (None, [C.POINTER(SgSolverOptions)]),
    "sg_device_options_default": (None, [C.POINTER(SgDeviceOptions)]),
    "sg_problem_from_map_frames": (C.c_int, [C.POINTER(SgMap), C.c_int32, C.c_int32, C.c_double,
                                             C.POINTER(SgProblem), C.POINTER(C.c_int32)]),
    "sg_problem_from_map_all": (C.c_int, [C.POINTER(SgMap), C.c_double, C.c_int32, C.POINTER(SgProblem),
                                          C.POINTER(C.c_int32)]),
    "sg_problem_free": (None, [C.POINTER(SgProblem)]),
    "sg_problem_write_back": (C.c_int, [C.POINTER(SgProblem), C.POINTER(SgMap)]),
    "sg_problem_shard": (C.c_int, [C.POINTER(SgProblem), C.c_int32, C.c_int32, C.POINTER(SgProblem)]),
    "sg_ba_create": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(SgDeviceOptions)]),
    "sg_ba_destroy": (None, [C.c_void_p]),
    "sg_comm_unique_id": (C.c_int, [C.c_void_p]),
    "sg_ba_comm_init": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32]),
    "sg_comm_group_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int32]),
    "sg_comm_group_destroy": (None, [C.c_void_p]),
    "sg_ba_comm_init_local": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32]),
    "sg_ba_comm_init_host": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "sg_ba_load": (C.c_int, [C.c_void_p, C.POINTER(SgProblem)]),
    "sg_ba_reserve": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32]),
    "sg_ba_load_counts": (C.c_int, [C.c_void_p, _ip, _ip]),
    "sg_ba_info_get": (C.c_int, [C.c_void_p, C.POINTER(SgBaInfo)]),
    "sg_ba_solve": (C.c_int, [C.c_void_p, C.POINTER(SgSolverOptions), C.POINTER(SgProblem),
                              C.POINTER(SgSolverSummary)]),
    "sg_ba_begin": (C.c_int, [C.c_void_p, C.POINTER(SgSolverOptions)]),
    "sg_ba_iterate": (C.c_int, [C.c_void_p, C.c_int32]),
    "sg_ba_sync": (C.c_int, [C.c_void_p]),
    "sg_ba_summary": (C.c_int, [C.c_void_p, C.POINTER(SgSolverSummary)]),
    "sg_ba_download": (C.c_int, [C.c_void_p, C.POINTER(SgProblem)]),
    "sg_ba_set_timing": (C.c_int, [C.c_void_p, C.c_int32]),
    "sg_ba_kernel_times": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int32, _dp, _ip, C.c_int32]),
    "sg_ba_kernel_work": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int32]),
    "sg_ba_evaluate": (C.c_int, [C.c_void_p, _dp, _dp, _ip]),
    "sg_ba_sweep": (C.c_int, [C.c_void_p, C.c_int32]),
    "sg_tracker_options_default": (None, [C.POINTER(SgTrackerOptions)]),
    "sg_tracker_create": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(SgTrackerOptions), C.POINTER(SgDeviceOptions)]),
    "sg_tracker_destroy": (None, [C.c_void_p]),
    "sg_tracker_set_image": (C.c_int, [C.c_void_p, C.c_int32, _u8p, C.c_int32, C.c_int32, C.c_int32]),
    "sg_tracker_get_level": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, _fp, _ip, _ip]),
    "sg_tracker_get_patches": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, _fp, _fp, _fp, _fp]),
    "sg_tracker_track": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, _fp, _fp, _ip, _ip, _ip]),
    "sg_tracker_load_features": (C.c_int, [C.c_void_p, C.c_int32, _fp, _fp, _ip]),
    "sg_tracker_run": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32]),
    "sg_tracker_results": (C.c_int, [C.c_void_p, _fp, _ip, _ip]),
    "sg_tracker_kernel_ms": (C.c_int, [C.c_void_p, _dp, _dp]),
    "sg_tracker_track_feature": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, _fp, _fp, _ip, _ip, _ip]),
    "sg_tracker_seed_features": (C.c_int, [C.c_void_p, C.c_int32, _fp, C.c_int32, C.c_int32, C.c_double, C.c_double,
                                           _fp, _ip, _fp, _ip]),
    "sg_matcher_create": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(SgDeviceOptions)]),
    "sg_matcher_destroy": (None, [C.c_void_p]),
    "sg_hamming_match": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32, C.POINTER(C.c_uint64), C.c_int32,
                                   _ip, _ip, _ip]),
    "sg_hamming_load": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32, C.POINTER(C.c_uint64), C.c_int32]),
    "sg_hamming_run": (C.c_int, [C.c_void_p, C.c_int32]),
    "sg_hamming_results": (C.c_int, [C.c_void_p, _ip, _ip, _ip, _dp]),
    "sg_slam_create": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(SgDeviceOptions)]),
    "sg_slam_destroy": (None, [C.c_void_p]),
    "sg_slam_solve_frames": (C.c_int, [C.c_void_p, C.POINTER(SgMap), C.c_int32, C.c_int32, C.c_double,
                                       C.POINTER(C.c_int32)]),
    "sg_slam_solve_all_frames": (C.c_int, [C.c_void_p, C.POINTER(SgMap), C.c_double, C.c_int32,
                                           C.POINTER(C.c_int32)]),
    "sg_slam_reproject_map": (C.c_int, [C.c_void_p, C.POINTER(SgMap), _dp]),
    "sg_map_clean": (C.c_int, [C.c_void_p, C.POINTER(SgMap), C.c_double, C.POINTER(C.c_int32)]),
    "sg_map_apply_epipolar": (C.c_int, [C.c_void_p, C.POINTER(SgMap), C.POINTER(C.c_int32)]),
    "sg_map_normalize": (C.c_int, [C.c_void_p, C.POINTER(SgMap)]),
    "sg_slam_iterations": (C.c_int32, [C.c_void_p]),
    "sg_slam_load_counts": (C.c_int, [C.c_void_p, _ip, _ip]),
    "sg_slam_last_phase_ms": (C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    "sg_slam_error": (C.c_double, [C.c_void_p]),
    "sg_slam_last_summary": (C.c_int, [C.c_void_p, C.POINTER(SgSolverSummary)]),
    "sg_slam_set_options": (C.c_int, [C.c_void_p, C.POINTER(SgSolverOptions)]),
    "sg_frontend_create": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(SgTrackerOptions), C.POINTER(SgDeviceOptions)]),
    "sg_frontend_destroy": (None, [C.c_void_p]),
    "sg_frontend_track": (C.c_int, [C.c_void_p, _u8p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                    C.POINTER(SgMapCallbacks), C.POINTER(C.c_int32), C.POINTER(SgFrontendStats)]),
    "sg_frontend_features": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
}


class SlamGpuError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH):
    """Load libslamgpu.so (the HIP build).  Raises if it is missing: the product has no CPU path."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise SlamGpuError(f"libslamgpu.so not built at {path}: run __graft_entry__.build() "
                           "(the HIP extension is required; there is no CPU fallback)")
    lib = C.CDLL(path)
    for name, (res, args) in SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(rc: int, what: str = ""):
    if rc != SG_OK:
        msg = _LIB.sg_last_error().decode() if _LIB is not None else ""
        raise SlamGpuError(f"{what} failed with code {rc}: {msg}")
