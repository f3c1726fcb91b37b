"""Developer diagnostics: device solver vs oracle on C1/C2 (prints, no asserts)."""
import os, sys, time, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle
from slamgpu.scene import make_config
from slamgpu import ba
from slamgpu.capi import default_solver_options

def run(name, nthreads=8):
    m = make_config(name)
    pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    po = oracle.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    print(name, "obs", pa.num_obs, "pts", pa.num_points, "frames", pa.num_frames, flush=True)
    same = all(np.array_equal(getattr(pa, f), getattr(po, f)) for f in pa.FIELDS)
    print("setup identical:", same, flush=True)
    g = ba.BundleAdjuster()
    g.load(pa)
    r, c, nf = g.evaluate()
    ro, co, nfo = oracle.evaluate(po.copy())
    print("evaluate: max|dr|", np.abs(r - ro).max(), "cost", c, co, "fail", nf, nfo, flush=True)
    t = time.time(); sg = g.solve(); tg = time.time() - t
    t = time.time(); so = oracle.solve(po, nthreads=nthreads); to = time.time() - t
    print("gpu   ", json.dumps(sg), "%.3fs" % tg, flush=True)
    print("oracle", json.dumps(so), "%.3fs" % to, flush=True)
    rg, cg, _ = oracle.evaluate(pa)
    rO, cO, _ = oracle.evaluate(po)
    print("final cost (oracle-eval) gpu %.9g oracle %.9g rel %.3e" % (cg, cO, abs(cg - cO) / cO))
    print("max |t diff|", np.abs(pa.t - po.t).max(), "max |q diff|", np.abs(pa.q - po.q).max())
    # iteration throughput (termination disabled)
    o = default_solver_options(max_num_iterations=1000000, disable_termination=1)
    g.load(pa); g.begin(o); g.iterate(5); g.sync()
    K = 50
    t = time.time(); g.iterate(K); g.sync(); dt = time.time() - t
    print("LM iterations/s: %.1f  (%.1f us/iter)" % (K / dt, 1e6 * dt / K), flush=True)
    g.set_timing(True); g.iterate(20); g.sync()
    for k, v in g.kernel_times().items(): print("   %-14s %8.1f us  n=%d" % (k, 1e3 * v[0], v[1]))
    g.set_timing(False)

if __name__ == "__main__":
    for name in sys.argv[1:] or ["C1"]:
        run(name)
