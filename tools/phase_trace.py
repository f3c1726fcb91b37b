"""Diagnostic: per-phase timeline of k_chol_tiles (SG_STAMP=1 build path): for each tile row K of the last
launch, the owner's chain (phase start -> (0) -> TRSM -> D update -> factor) and the latest wave's barrier
arrival, in s_memtime cycles relative to the phase start.  Usage: phase_trace.py [C2|C5]"""
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
g.iterate(5)
g.sync()
n = 64 + 2 * 128 * 16
buf = (C.c_ulonglong * n)()
g.lib.sg_ba_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
g.lib.sg_ba_debug_stamps(g.h, buf, n)
nt = (info["n"] + 15) // 16
nd = info["cholesky_split"]
print("config %s n=%d NT=%d split=%d" % (name, info["n"], nt, nd))
for wg in (0, 1) if nd else (0,):
    kmax = (nd if wg else (nt - nd - 7 + 7 if nd else nt))
    print("workgroup %d: K | owner: (0) trsm Dupd factor post->bar | last barrier arrival | phase" % wg)
    tot = [0] * 6
    prev_end = None
    for K in range(min(kmax, 128)):
        row = [buf[64 + (wg * 128 + K) * 16 + s] for s in range(16)]
        st, a0, a1, a2, a3 = row[8:13]
        bar = max(row[0:8])
        own_bar = None
        if st == 0:
            continue
        seg = [a0 - st, a1 - a0, a2 - a1, a3 - a2, bar - a3]
        ph = (bar - prev_end) if prev_end else None
        prev_end = bar
        for i, v in enumerate(seg):
            tot[i] += v
        print("  K=%3d  %6d %6d %6d %6d %6d   phase %s" % (K, *seg, ph))
    print("  sum    %6d %6d %6d %6d %6d" % tuple(tot[:5]))
