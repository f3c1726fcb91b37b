"""Python mirror of the reference's Slam interface (slam.h:21-65) over libslamgpu.so.

`Slam` keeps the reference's method names and semantics (SolveFrames / SolveAllFrames / ReprojectMap,
iterations(), error()); `BundleAdjuster` exposes the device solver directly for benchmarks and the
landmark-sharded multi-GPU path.  All compute runs in the HIP library; these classes only marshal.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .capi import (ProblemArrays, SgBaInfo, SgDeviceOptions, SgProblem, SgSolverOptions, SgSolverSummary,
                   check, default_solver_options, load_library)
from .scene import MapArrays


def _dev(device=0, precision=0, rank=0, nranks=1):
    return SgDeviceOptions(device=device, precision=precision, rank=rank, nranks=nranks)


def problem_from_map_frames(m: MapArrays, num_to_solve: int, num_to_present: int, range_: float = 2.0):
    """Slam::SolveFrames selection + SetupProblem (slam.cpp:257-443) -> ProblemArrays, or None on abort."""
    lib = load_library()
    p = SgProblem()
    built = C.c_int32()
    ms = m.struct()
    check(lib.sg_problem_from_map_frames(C.byref(ms), num_to_solve, num_to_present, range_, C.byref(p),
                                         C.byref(built)), "sg_problem_from_map_frames")
    if not built.value:
        return None
    pa = ProblemArrays.from_struct(p)
    lib.sg_problem_free(C.byref(p))
    return pa


def problem_from_map_all(m: MapArrays, range_: float = 2.0, solve_cameras: bool = False):
    lib = load_library()
    p = SgProblem()
    built = C.c_int32()
    ms = m.struct()
    check(lib.sg_problem_from_map_all(C.byref(ms), range_, int(solve_cameras), C.byref(p), C.byref(built)),
          "sg_problem_from_map_all")
    if not built.value:
        return None
    pa = ProblemArrays.from_struct(p)
    lib.sg_problem_free(C.byref(p))
    return pa


def shard_problem(pa: ProblemArrays, rank: int, nranks: int) -> ProblemArrays:
    """Landmark shard `rank` of `nranks` (points split by first observing frame; frames replicated)."""
    lib = load_library()
    out = SgProblem()
    ps = pa.struct()
    check(lib.sg_problem_shard(C.byref(ps), rank, nranks, C.byref(out)), "sg_problem_shard")
    sh = ProblemArrays.from_struct(out)
    lib.sg_problem_free(C.byref(out))
    return sh


class LocalCommGroup:
    """sg_comm_group: nranks solver handles on one device exchanging in-process instead of over RCCL."""

    def __init__(self, nranks: int):
        self.lib = load_library()
        self.h = C.c_void_p()
        check(self.lib.sg_comm_group_create(C.byref(self.h), nranks), "sg_comm_group_create")

    def close(self):
        if self.h:
            self.lib.sg_comm_group_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BundleAdjuster:
    """The device solver (sg_ba): load a problem, solve or run fixed LM iterations."""

    def __init__(self, device: int = 0, precision: int = 0):
        self.lib = load_library()
        self.h = C.c_void_p()
        dev = _dev(device, precision)
        check(self.lib.sg_ba_create(C.byref(self.h), C.byref(dev)), "sg_ba_create")
        self._pa = None

    def close(self):
        if self.h:
            self.lib.sg_ba_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = C.create_string_buffer(uid, 128)
        check(self.lib.sg_ba_comm_init(self.h, buf, nranks, rank), "sg_ba_comm_init")

    def comm_init_local(self, group: "LocalCommGroup", rank: int):
        """Join an in-process communicator group (one device, one host thread per rank; tests)."""
        check(self.lib.sg_ba_comm_init_local(self.h, group.h, rank), "sg_ba_comm_init_local")

    def comm_init_host(self, nranks: int, rank: int, allreduce):
        """Join a host-transport communicator (sg_ba_comm_init_host): allreduce(array, op) receives each of the
        solver's all-reduce buffers as a float64 numpy view of pinned host memory (op "sum" or "max") and
        reduces it in place across the ranks (e.g. torch.distributed over gloo, one process per rank)."""
        import numpy as np
        from .capi import ALLREDUCE_FN

        def cb(buf, n, op, user):
            try:
                allreduce(np.ctypeslib.as_array(buf, shape=(int(n),)), "max" if op == 1 else "sum")
                return 0
            except Exception:   # noqa: BLE001 - reported to the solver as SG_ECOMM
                return 1
        self._allreduce_cb = ALLREDUCE_FN(cb)   # kept alive as long as the handle
        check(self.lib.sg_ba_comm_init_host(self.h, nranks, rank, C.cast(self._allreduce_cb, C.c_void_p), None),
              "sg_ba_comm_init_host")

    @staticmethod
    def unique_id() -> bytes:
        lib = load_library()
        buf = C.create_string_buffer(128)
        check(lib.sg_comm_unique_id(buf), "sg_comm_unique_id")
        return buf.raw

    def load(self, pa: ProblemArrays):
        self._pa = pa
        ps = pa.struct()
        check(self.lib.sg_ba_load(self.h, C.byref(ps)), "sg_ba_load")

    def reserve(self, max_frames: int, max_points: int, max_obs: int):
        """Pre-size the device / pinned buffers for problems up to this size (drops the loaded problem if it
        reallocates)."""
        check(self.lib.sg_ba_reserve(self.h, max_frames, max_points, max_obs), "sg_ba_reserve")

    def load_counts(self) -> tuple:
        """(full loads, value-only loads): a load with the previous load's structure reuses its index lists."""
        full, vals = C.c_int32(0), C.c_int32(0)
        check(self.lib.sg_ba_load_counts(self.h, C.byref(full), C.byref(vals)), "sg_ba_load_counts")
        return full.value, vals.value

    def info(self) -> dict:
        """What the last load set up: sizes, Cholesky band and path, Schur pair count, shard."""
        i = SgBaInfo()
        check(self.lib.sg_ba_info_get(self.h, C.byref(i)), "sg_ba_info_get")
        return i.as_dict()

    def solve(self, options: SgSolverOptions = None) -> dict:
        o = options or default_solver_options()
        s = SgSolverSummary()
        ps = self._pa.struct()
        check(self.lib.sg_ba_solve(self.h, C.byref(o), C.byref(ps), C.byref(s)), "sg_ba_solve")
        return s.as_dict()

    def begin(self, options: SgSolverOptions):
        check(self.lib.sg_ba_begin(self.h, C.byref(options)), "sg_ba_begin")

    def iterate(self, n: int):
        check(self.lib.sg_ba_iterate(self.h, n), "sg_ba_iterate")

    def sweep(self, n: int):
        """n Jacobian/Hessian sweeps (k_linearize) at the current state — benchmark of the HBM kernel."""
        check(self.lib.sg_ba_sweep(self.h, n), "sg_ba_sweep")

    def sync(self):
        check(self.lib.sg_ba_sync(self.h), "sg_ba_sync")

    def summary(self) -> dict:
        s = SgSolverSummary()
        check(self.lib.sg_ba_summary(self.h, C.byref(s)), "sg_ba_summary")
        return s.as_dict()

    def download(self):
        ps = self._pa.struct()
        check(self.lib.sg_ba_download(self.h, C.byref(ps)), "sg_ba_download")

    def evaluate(self):
        n = self._pa.num_obs
        r = np.zeros(2 * n)
        cost = C.c_double()
        nf = C.c_int32()
        check(self.lib.sg_ba_evaluate(self.h, r.ctypes.data_as(C.POINTER(C.c_double)), C.byref(cost),
                                      C.byref(nf)), "sg_ba_evaluate")
        return r.reshape(-1, 2), cost.value, nf.value

    def set_timing(self, on: bool):
        check(self.lib.sg_ba_set_timing(self.h, int(on)), "sg_ba_set_timing")

    def kernel_times(self) -> dict:
        names = C.create_string_buffer(1024)
        ms = np.zeros(32)
        cnt = np.zeros(32, dtype=np.int32)
        check(self.lib.sg_ba_kernel_times(self.h, names, 1024, ms.ctypes.data_as(C.POINTER(C.c_double)),
                                          cnt.ctypes.data_as(C.POINTER(C.c_int32)), 32), "sg_ba_kernel_times")
        nm = names.value.decode().split(",")
        return {n: (float(ms[i]), int(cnt[i])) for i, n in enumerate(nm)}

    def kernel_work(self) -> dict:
        by = np.zeros(32)
        fl = np.zeros(32)
        check(self.lib.sg_ba_kernel_work(self.h, by.ctypes.data_as(C.POINTER(C.c_double)),
                                         fl.ctypes.data_as(C.POINTER(C.c_double)), 32), "sg_ba_kernel_work")
        names = ["linearize", "cam_reduce", "cam_finalize", "schur", "S_reduce", "cholesky", "point_update",
                 "upd_reduce", "decide"]
        out = {n: (float(by[i]), float(fl[i])) for i, n in enumerate(names)}
        # derived figures after the kernels' slots (KernelWork, ba_solver.hip): k_schur's useful flops (no zero
        # tiles) and SURVEY 8d's algorithmic bytes of one linearization sweep at f64
        out["schur_useful"] = (0.0, float(fl[10]))
        out["sweep_survey_model"] = (float(by[11]), 0.0)
        return out


class Slam:
    """slam.h:21-65 — the reference's Slam object, backed by the MI355X solver."""

    def __init__(self, device: int = 0, options: SgSolverOptions = None):
        self.lib = load_library()
        self.h = C.c_void_p()
        dev = _dev(device)
        check(self.lib.sg_slam_create(C.byref(self.h), C.byref(dev)), "sg_slam_create")
        if options is not None:
            check(self.lib.sg_slam_set_options(self.h, C.byref(options)), "sg_slam_set_options")

    def __del__(self):
        try:
            if self.h:
                self.lib.sg_slam_destroy(self.h)
        except Exception:
            pass

    def SolveFrames(self, m: MapArrays, num_to_solve: int, num_to_present: int, range_: float) -> bool:
        solved = C.c_int32()
        ms = m.struct()
        check(self.lib.sg_slam_solve_frames(self.h, C.byref(ms), num_to_solve, num_to_present, range_,
                                            C.byref(solved)), "Slam::SolveFrames")
        return bool(solved.value)

    def SolveAllFrames(self, m: MapArrays, range_: float, solve_cameras: bool) -> bool:
        solved = C.c_int32()
        ms = m.struct()
        check(self.lib.sg_slam_solve_all_frames(self.h, C.byref(ms), range_, int(solve_cameras),
                                                C.byref(solved)), "Slam::SolveAllFrames")
        return bool(solved.value)

    def SolveFramePose(self, f1, f2) -> bool:
        """slam.cpp:180-182: the reference returns false unconditionally (dead code after the return)."""
        return False

    def ReprojectMap(self, m: MapArrays) -> float:
        mean = C.c_double()
        ms = m.struct()
        check(self.lib.sg_slam_reproject_map(self.h, C.byref(ms), C.byref(mean)), "Slam::ReprojectMap")
        return mean.value

    # LocalMap maintenance (localmap.cpp), on the device through the same handle.  These mirror
    # LocalMap::Clean / LocalMap::ApplyEpipolarConstraint, which main.cpp calls after each solve.
    def Clean(self, m: MapArrays, error_threshold: float) -> bool:
        """LocalMap::Clean (localmap.cpp:283-398) on m's ReprojectMap residuals; mutates m in place."""
        res = C.c_int32()
        ms = m.struct()
        check(self.lib.sg_map_clean(self.h, C.byref(ms), error_threshold, C.byref(res)), "LocalMap::Clean")
        return bool(res.value)

    def ApplyEpipolarConstraint(self, m: MapArrays) -> int:
        """LocalMap::ApplyEpipolarConstraint (localmap.cpp:232-276); mutates m.  Returns the violation count."""
        n = C.c_int32()
        ms = m.struct()
        check(self.lib.sg_map_apply_epipolar(self.h, C.byref(ms), C.byref(n)), "LocalMap::ApplyEpipolarConstraint")
        return n.value

    def Normalize(self, m: MapArrays):
        """LocalMap::Normalize (localmap.cpp:114-155) on the device; mutates m's poses and points in place."""
        ms = m.struct()
        check(self.lib.sg_map_normalize(self.h, C.byref(ms)), "LocalMap::Normalize")

    def iterations(self) -> int:
        return int(self.lib.sg_slam_iterations(self.h))

    def load_counts(self) -> tuple:
        """(full loads, value-only loads) of SolveFrames / SolveAllFrames calls on this object."""
        full, vals = C.c_int32(0), C.c_int32(0)
        check(self.lib.sg_slam_load_counts(self.h, C.byref(full), C.byref(vals)), "sg_slam_load_counts")
        return full.value, vals.value

    def last_phase_ms(self) -> dict:
        """Host wall time of the last SolveFrames / SolveAllFrames call by phase (ms)."""
        v = (C.c_double * 4)()
        check(self.lib.sg_slam_last_phase_ms(self.h, v), "sg_slam_last_phase_ms")
        return {"setup": v[0], "load": v[1], "solve": v[2], "write_back": v[3]}

    def error(self) -> float:
        return float(self.lib.sg_slam_error(self.h))

    def last_summary(self) -> dict:
        s = SgSolverSummary()
        check(self.lib.sg_slam_last_summary(self.h, C.byref(s)), "sg_slam_last_summary")
        return s.as_dict()
