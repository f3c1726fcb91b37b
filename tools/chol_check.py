"""Diagnostic: two solves per setting (default, deterministic Schur sums, window Cholesky): bitwise reproducibility."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, json, numpy as np
sys.path.insert(0, "%s/slam-robot_amd")
from slamgpu import ba
from slamgpu.scene import make_config
m = make_config(sys.argv[1])
pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
out = []
for rep in range(2):
    g = ba.BundleAdjuster(); p = pa.copy(); g.load(p); s = g.solve()
    out.append([s["num_iterations"], s["final_cost"].hex(), float(np.abs(p.t).sum()).hex()])
print(json.dumps(out))
''' % ROOT
for cfg in sys.argv[1:] or ["C2"]:
    for env in ({}, {"SG_DETERMINISTIC": "1"}, {"SG_CHOL_WINDOW": "1", "SG_DETERMINISTIC": "1"}):
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, "-c", code, cfg], env=e, capture_output=True, text=True)
        print(cfg, env, r.stdout.strip() or r.stderr[-500:])
