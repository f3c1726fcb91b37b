"""Diagnostic (round 6): k_chol_tiles barrier arrivals per column offset d = J - K (d = 0: the late wave, 1: the
owner of the phase, 2: the next owner, ...), from a -DSG_X_ARRIVE build of ba_chol.hip (tools/build_variant.sh) run
with SG_STAMP=1: mean and max cycles from a wave's phase start (barrier exit) to its barrier arrival, per workgroup.
Usage: SG_LIB_PATH=<variant .so> arrive_trace.py [C2|C5]"""
import ctypes as C
import os
import sys

os.environ["SG_STAMP"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
from slamgpu import ba  # noqa: E402
from slamgpu.capi import default_solver_options  # noqa: E402
from slamgpu.scene import make_config  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
m = make_config(name)
pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
g = ba.BundleAdjuster()
g.load(pa)
info = g.info()
g.begin(default_solver_options(max_num_iterations=10 ** 6, disable_termination=1, always_linearize=1))
g.iterate(10)
g.sync()
KSEG = 64 + 2 * 128 * 16 + 16
n = KSEG + 512 + 2 * 256
buf = (C.c_ulonglong * n)()
g.lib.sg_ba_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
g.lib.sg_ba_debug_stamps(g.h, buf, n)
print("config %s n=%d split=%d" % (name, info["n"], info["cholesky_split"]))
for wg in (0, 1):
    tot = [0] * 8
    mx = [0] * 8
    cnt = [0] * 8
    for w in range(8):
        o = KSEG + wg * 256 + w * 24
        for q in range(8):
            tot[q] += buf[o + q]
            mx[q] = max(mx[q], buf[o + 8 + q])
            cnt[q] += buf[o + 16 + q]
    if sum(cnt) == 0:
        continue
    print("workgroup %d: d | phases | mean arrival | max arrival (cycles from the phase start)" % wg)
    for q in range(8):
        if cnt[q]:
            print("  d=%d  %6d  %8.0f  %8d" % (q, cnt[q], tot[q] / cnt[q], mx[q]))
    st = [sum(buf[KSEG + 512 + wg * 256 + w * 16 + s] for w in range(8)) for s in range(16)]
    nl, no, nx = cnt[0], cnt[1], sum(cnt[2:])
    print("  late  (per late phase):  W mfma %.0f | loads %.0f | W store %.0f | z' %.0f | -> arrival %.0f" %
          tuple(st[i] / max(nl, 1) for i in range(5)))
    print("  owner (per owner phase): (0) %.0f | TRSM %.0f | Dupd %.0f | tile_diag %.0f | -> arrival %.0f" %
          tuple(st[i] / max(no, 1) for i in range(5, 10)))
    print("  other (per wave-phase):  (0) %.0f | TRSM %.0f | W %.0f | -> arrival %.0f" %
          tuple(st[i] / max(nx, 1) for i in range(10, 14)))
