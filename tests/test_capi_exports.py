"""The C-ABI library loads (no GPU needed) and exports every symbol include/slamgpu.h declares."""
import ctypes as C
import os
import re

from slamgpu.capi import LIB_PATH, SgDeviceOptions, SgSolverOptions, default_solver_options, load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sg_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB_PATH), "build libslamgpu.so first (__graft_entry__.build())"
    lib = C.CDLL(LIB_PATH)
    names = _declared("slamgpu.h")
    assert len(names) > 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_host_only_entry_points_work_without_a_gpu():
    lib = load_library()
    assert b"gfx950" in lib.sg_version()
    o = SgSolverOptions()
    lib.sg_solver_options_default(C.byref(o))
    ref = default_solver_options()
    for name, _ in SgSolverOptions._fields_:
        assert getattr(o, name) == getattr(ref, name), name
    d = SgDeviceOptions()
    lib.sg_device_options_default(C.byref(d))
    assert (d.device, d.precision, d.rank, d.nranks) == (0, 0, 0, 1)


def test_null_arguments_return_einval():
    lib = load_library()
    assert lib.sg_ba_load(None, None) == -22
    assert lib.sg_problem_write_back(None, None) == -22
    full, vals = C.c_int32(7), C.c_int32(7)
    assert lib.sg_ba_load_counts(None, C.byref(full), C.byref(vals)) == -22
    assert lib.sg_slam_load_counts(None, C.byref(full), C.byref(vals)) == -22
    assert lib.sg_last_error()
