"""End-to-end Slam::SolveFrames timing at config 2 (host problem setup + upload + device LM solve + write-back)
next to the device-only LM iterations, to size the host share of a real call."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
from slamgpu import ba  # noqa: E402
from slamgpu.capi import default_solver_options  # noqa: E402
from slamgpu.scene import make_scene  # noqa: E402

m = make_scene(num_frames=50, num_points=20000, seed=2, run_max=14)
slam = ba.Slam(device=0)
slam.SolveFrames(m.copy(), 48, 50, 2.0)   # warm up (allocations, code objects); later calls reuse its structure
reps = 5
t_build = t_load = 0.0
for _ in range(reps):
    t0 = time.perf_counter()
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    t1 = time.perf_counter()
    g = ba.BundleAdjuster(device=0)
    g.load(pa)
    g.sync()
    t2 = time.perf_counter()
    t_build += t1 - t0
    t_load += t2 - t1
    g.close()
tot, its = 0.0, 0
for _ in range(reps):
    mm = m.copy()
    it0 = slam.iterations()
    t0 = time.perf_counter()
    slam.SolveFrames(mm, 48, 50, 2.0)
    tot += time.perf_counter() - t0
    its += slam.iterations() - it0
print("SolveFrames end to end: %.2f ms per call, %.1f LM iterations per call (%.3f ms per iteration incl. setup)"
      % (1e3 * tot / reps, its / reps, 1e3 * tot / max(its, 1)))
print("  host SetupProblem (sg_problem_from_map_frames): %.2f ms; sg_ba_load (work lists + upload): %.2f ms"
      % (1e3 * t_build / reps, 1e3 * t_load / reps))
t_solve = 0.0
for _ in range(reps):
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    g = ba.BundleAdjuster(device=0)
    g.load(pa)
    g.sync()
    t0 = time.perf_counter()
    sm = g.solve()
    t_solve += time.perf_counter() - t0
    g.close()
print("  sg_ba_solve (LM loop, polling every 8 iterations, + download): %.2f ms for %d iterations"
      % (1e3 * t_solve / reps, sm["num_iterations"]))
# incremental update: loads on one handle with an unchanged structure re-upload the values only
g = ba.BundleAdjuster(device=0)
g.load(ba.problem_from_map_frames(m, 48, 50, 2.0))
t_val = 0.0
for _ in range(reps):
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    t0 = time.perf_counter()
    g.load(pa)
    g.sync()
    t_val += time.perf_counter() - t0
print("  sg_ba_load, same structure as the previous load (values only): %.2f ms; loads (full, values) %s"
      % (1e3 * t_val / reps, g.load_counts()))
print("  Slam object loads (full, values): %s" % (slam.load_counts(),))
g.close()
