"""Diagnostic: per-phase cycle breakdown of stamped kernels (SG_STAMP=1)."""
import ctypes as C, os, sys, time
os.environ["SG_STAMP"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
import numpy as np
from slamgpu import ba
from slamgpu.capi import default_solver_options
from slamgpu.scene import make_config
name = sys.argv[1] if len(sys.argv) > 1 else "C2"
m = make_config(name)
pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
g = ba.BundleAdjuster(); g.load(pa)
g.begin(default_solver_options(max_num_iterations=10**6, disable_termination=1))
N = 20
g.iterate(N); g.sync()
buf = (C.c_ulonglong * 64)()
g.lib.sg_ba_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
g.lib.sg_ba_debug_stamps(g.h, buf, 64)
names = ["initial window load", "prefetch+panel load", "panel stores+barrier", "panel factor loop", "trailing update",
         "slide", "xc/y stores+sync", "candidates", "last W pass", "W sync", "backsub loop rest",
         "bs load wait+fma", "bs dpp reduce", "bs store+barrier", "loop head+prefetch issue", "panel column loads"]
tot = sum(buf[i] for i in range(len(names)))
for i, n in enumerate(names):
    print("%-18s %10.0f cycles/iter  (%4.1f%%)" % (n, buf[i] / N, 100.0 * buf[i] / max(tot, 1)))
print("total %.0f cycles/iter" % (tot / N))
