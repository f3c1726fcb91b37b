"""A/B of the tiled Cholesky's variants (env switches read when a handle is created) in one process: for each
variant a fresh handle on C2 (and C5), per-kernel HIP-event times over always-linearize iterations, and an
8-iteration solve from the perturbed start compared with the first variant's (cost, poses).
Usage: chol_ab.py [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
import numpy as np  # noqa: E402

from slamgpu import ba  # noqa: E402
from slamgpu.capi import default_solver_options  # noqa: E402
from slamgpu.scene import make_config  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
VARIANTS = [
    ("la", {"SG_CHOL_LOOKAHEAD": "1", "SG_CHOL_FACTOR": "0", "SG_CHOL_DINV": "0", "SG_CHOL_DATAFLOW": "0"}),
    ("la+df", {"SG_CHOL_LOOKAHEAD": "1", "SG_CHOL_FACTOR": "0", "SG_CHOL_DINV": "0", "SG_CHOL_DATAFLOW": "1"}),
    ("base", {"SG_CHOL_LOOKAHEAD": "0", "SG_CHOL_FACTOR": "0", "SG_CHOL_DINV": "0", "SG_CHOL_DATAFLOW": "0"}),
]
out = {}
for cfg in ("C2", "C5"):
    m = make_config(cfg)
    pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    ref = None
    for name, env in VARIANTS:
        os.environ.update(env)
        g = ba.BundleAdjuster()
        p = pa.copy()
        g.load(p)
        s = g.solve(default_solver_options(max_num_iterations=8))
        if ref is None:
            ref = (s, p.q.copy(), p.t.copy())
        dcost = abs(s["final_cost"] - ref[0]["final_cost"]) / ref[0]["final_cost"]
        dq = float(np.abs(p.q - ref[1]).max())
        dt = float(np.abs(p.t - ref[2]).max())
        same = s["num_successful_steps"] == ref[0]["num_successful_steps"] and s["sync_timeouts"] == 0
        g.load(pa.copy())
        g.begin(default_solver_options(max_num_iterations=10 ** 6, disable_termination=1, always_linearize=1))
        g.iterate(5)
        g.sync()
        t0 = time.perf_counter()
        g.iterate(steps)
        g.sync()
        wall = (time.perf_counter() - t0) / steps * 1e3
        g.set_timing(True)
        g.iterate(steps)
        g.sync()
        kt = g.kernel_times()
        summ = g.summary()
        g.close()
        ch = kt.get("cholesky", (0, 0))[0] * 1e3
        res = {"ms_per_iter": wall, "chol_us": ch, "kernels_us": {k: round(v[0] * 1e3, 2) for k, v in kt.items()},
               "solve_dcost": dcost, "solve_dq": dq, "solve_dt": dt, "same_steps": same,
               "timeouts": summ["sync_timeouts"]}
        out["%s/%s" % (cfg, name)] = res
        print("%s %-12s iter %.4f ms  chol %.1f us  dcost %.1e dq %.1e dt %.1e same %s tmo %d" % (
            cfg, name, wall, ch, dcost, dq, dt, same, summ["sync_timeouts"]), flush=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "chol_ab.json"), "w"), indent=1)
