"""Diagnostic: per-phase cycle breakdown of k_chol_tiles (SG_STAMP=1): lane 0 of waves 0 (slots 0-7) and
1 (slots 8-15), cycles per LM iteration."""
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
fac = ["init load/factor", "init sync", "phase tail (W,reload)", "phase barrier", "W sync", "backsub",
       "tail+cand", "bs compute", "(0) trailing", "(1) trsm", "(2) D update", "(2) factor", "(3) W",
       "(4) reload", "bs barrier", "bs sum"]
col = fac
print("config %s n=%d" % (name, 6 * (m.num_frames - 2)))
for i in range(16):
    print("wave0 %-22s %9.0f   wave1 %9.0f" % (fac[i], buf[i] / N, buf[16 + i] / N))
print("total wave0 %.0f  wave1 %.0f cycles/iter" % (sum(buf[:16]) / N, sum(buf[16:32]) / N))
