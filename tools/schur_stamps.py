"""Diagnostic: per-phase cycle breakdown of k_schur's workgroup 0 (SG_STAMP=1): producer wave 0 (slots 32-36)
and consumer wave 4 (slots 40-45), cycles per LM iteration, plus the segment's batch count."""
import ctypes as C, os, sys
os.environ["SG_STAMP"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
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
names = {32: "P prologue points", 33: "P prologue barrier", 34: "P cells", 35: "P points", 36: "P barrier",
         40: "C prologue", 41: "C prologue barrier", 42: "C mfma", 44: "C barrier", 45: "C store"}
print("config %s" % name)
for k, v in names.items():
    print("%-22s %10.0f" % (v, buf[k] / N))
