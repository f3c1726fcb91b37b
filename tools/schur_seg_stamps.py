"""Diagnostic: per-segment cycles of k_schur (a library built with -DSG_SEG_STAMPS, tools/build_variant.sh,
loaded through SG_LIB_PATH): for every segment its workgroup span and the busy cycles (work between barriers) of
the first cell wave, the point wave and the first MFMA wave, summed over N iterations, with its point range and
batch count.  Usage: schur_seg_stamps.py <config> <out.json>"""
import ctypes as C, json, os, sys
os.environ["SG_STAMP"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
from slamgpu import ba
from slamgpu.capi import default_solver_options
from slamgpu.scene import make_config
name, out = sys.argv[1], sys.argv[2]
m = make_config(name)
pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
g = ba.BundleAdjuster(); g.load(pa)
g.begin(default_solver_options(max_num_iterations=10**6, disable_termination=1))
N = 10
g.iterate(N); g.sync()
KSEG = 64 + 2 * 128 * 16 + 16
n = KSEG + 8 * 1024
buf = (C.c_ulonglong * n)()
g.lib.sg_ba_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
g.lib.sg_ba_debug_stamps(g.h, buf, n)
segs = []
for k in range(1024):
    w = [buf[KSEG + 8 * k + i] for i in range(8)]
    if w[7] == 0:
        continue
    segs.append({"seg": k, "span": w[0] / w[7], "cells": w[1] / w[7], "points": w[2] / w[7], "mfma": w[3] / w[7],
                 "p0": w[4], "p1": w[5], "nbt": w[6], "launches": w[7]})
json.dump({"config": name, "env_equal": bool(os.environ.get("SG_SEG_EQUAL")), "segs": segs}, open(out, "w"))
sp = sorted(s["span"] for s in segs)
print(name, "equal" if os.environ.get("SG_SEG_EQUAL") else "balanced", "nseg", len(segs), "span max %.0f median %.0f min %.0f" % (sp[-1], sp[len(sp) // 2], sp[0]))
