"""Bitwise comparison of two in-tree library builds on the same problems (a refactor that must not change a bit).

Usage: python tools/lib_bitcmp.py <lib_a.so> <lib_b.so>.  Each build runs in its own process (SG_LIB_PATH is read
at import) on C2 (48, 50) and C5 (198, 200) in the benchmark regime (20 + 40 iterations, rejections included)
and in a solve to convergence, both with one and two waves per chunk; the poses, points and summaries must agree
bit for bit.
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, os
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "slam-robot_amd"))
from slamgpu import ba
from slamgpu.capi import default_solver_options
from slamgpu.scene import make_config
out = {}
arrs = {}
for cfg, lo, hi in (("C2", 48, 50), ("C5", 198, 200)):
    m = make_config(cfg)
    pa = ba.problem_from_map_frames(m, lo, hi, 2.0)
    for waves in ("1", "2"):
        os.environ["SG_LIN_WAVES"] = waves
        for regime in ("bench", "solve"):
            p = pa.copy()
            g = ba.BundleAdjuster()
            g.load(p)
            if regime == "solve":
                s = g.solve(None)
            else:
                g.begin(default_solver_options(max_num_iterations=10 ** 6, disable_termination=1, always_linearize=1))
                g.iterate(20)
                g.iterate(40)
                g.sync()
                s = g.summary()
                g.download()
            g.close()
            key = "%s_w%s_%s" % (cfg, waves, regime)
            out[key] = {k: v for k, v in s.items() if not k.endswith("_ms") and "time" not in k}
            arrs[key + "_q"] = p.q
            arrs[key + "_t"] = p.t
            arrs[key + "_X"] = p.X
np.savez(sys.argv[2] + ".npz", **arrs)
open(sys.argv[2] + ".json", "w").write(json.dumps(out, default=float))
"""


def run(lib, tag):
    env = dict(os.environ, SG_LIB_PATH=os.path.abspath(lib))
    dst = os.path.join(ROOT, "gpurun_out", "bitcmp_" + tag)
    subprocess.run([sys.executable, "-c", CHILD, ROOT, dst], env=env, check=True, timeout=300)
    return json.load(open(dst + ".json")), np.load(dst + ".npz")


def main():
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    sa, aa = run(sys.argv[1], "a")
    sb, ab = run(sys.argv[2], "b")
    bad = 0
    for k in sorted(sa):
        same_s = sa[k] == sb[k]
        same_a = all(np.array_equal(aa[k + s], ab[k + s]) for s in ("_q", "_t", "_X"))
        print("%-16s summary %s arrays %s  (iterations %s, cost %r)" % (
            k, "same" if same_s else "DIFF", "same" if same_a else "DIFF", sa[k].get("num_iterations"),
            sa[k].get("final_cost")))
        if not same_s:
            print("   a:", {x: sa[k][x] for x in sa[k] if sa[k][x] != sb[k].get(x)})
            print("   b:", {x: sb[k].get(x) for x in sa[k] if sa[k][x] != sb[k].get(x)})
        bad += (not same_s) + (not same_a)
    print("bitcmp", "OK" if bad == 0 else "FAILED (%d)" % bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
