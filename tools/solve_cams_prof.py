"""SolveAllFrames(C2 map, 2.0, solve_cameras) iterations for a rocprofv3 kernel trace: the bordered band solve
(k_chol_tiles + k_chol_border) against SG_CHOL_BORDER=0's k_cholesky_global.  Usage: solve_cams_prof.py [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
from slamgpu import ba  # noqa: E402
from slamgpu.capi import default_solver_options  # noqa: E402
from slamgpu.scene import make_config  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
p = ba.problem_from_map_all(make_config("C2"), 2.0, True)
g = ba.BundleAdjuster()
g.load(p)
g.begin(default_solver_options(max_num_iterations=steps + 8, disable_termination=1, always_linearize=1))
g.iterate(steps)
g.sync()
s = g.summary()
print(g.info()["cholesky"], s["num_lm_iterations"], s["ok"], flush=True)
if os.environ.get("SG_STAMP") == "1":   # k_chol_border's per-step s_memtime sums (d.stamps[48..56])
    import ctypes as C
    import numpy as np
    buf = np.zeros(64, np.uint64)
    g.lib.sg_ba_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    g.lib.sg_ba_debug_stamps(g.h, buf.ctypes.data, 64)
    names = ["chain", "C solve", "z'", "back-sub", "end", "after B1", "after B2", "after B3", "after B4"]
    t = {k: round(float(buf[48 + i]) / steps) for i, k in enumerate(names)}
    order = ["chain", "after B1", "after B2", "C solve", "after B3", "z'", "after B4", "back-sub", "end"]
    print("k_chol_border, ticks from its start (per launch):", [(k, t[k]) for k in order], flush=True)
    print("k_intr_fk<0>, <1> mid-grid workgroup (loop, sums, tail ticks):",
          [round(float(buf[58 + i]) / steps) for i in range(6)], flush=True)
g.close()
