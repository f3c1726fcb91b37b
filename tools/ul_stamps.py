"""Diagnostic: per-step cycle breakdown of k_update_lin (SG_STAMP=1): lane 0 of the mid-grid and of the last
workgroup, s_memtime cycles per launch for each step of a round (pass 1, pass 2, candidate observations, point
blocks, unit scalars, the final stores)."""
import ctypes as C, os, sys
os.environ["SG_STAMP"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
from slamgpu import ba
from slamgpu.capi import default_solver_options
from slamgpu.scene import make_config
K_UL = 64 + 2 * 128 * 16   # kUlStamp in ba_solver.hip
names = ["pass1 (A_p^T A_c x_c)", "pass2 (point step)", "candidate observations", "point blocks",
         "unit scalars", "final stores"]
for name in (sys.argv[1:] or ["C2", "C5"]):
    m = make_config(name)
    pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    g = ba.BundleAdjuster(); g.load(pa)
    g.begin(default_solver_options(max_num_iterations=10**6, disable_termination=1))
    g.iterate(20); g.sync()
    n = K_UL + 16
    buf = (C.c_ulonglong * n)()
    g.lib.sg_ba_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    g.lib.sg_ba_debug_stamps(g.h, buf, n)
    for w, wn in ((0, "mid-grid"), (1, "last")):
        L = max(1, buf[K_UL + 8 * w + 6])
        row = ["%s %.0f" % (nm, buf[K_UL + 8 * w + k] / L) for k, nm in enumerate(names)]
        print("%s %s workgroup (%d launches, s_memtime cycles per launch): %s" % (name, wn, L, "; ".join(row)))
