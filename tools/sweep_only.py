"""Profiling driver: the scaled Jacobian sweep alone (k_linearize on a ~1.65M-observation problem), for
rocprofv3 kernel traces and PMC passes.  Prints the HIP-event launch time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
from slamgpu import ba  # noqa: E402
from slamgpu.capi import default_solver_options  # noqa: E402
from slamgpu.scene import make_scene  # noqa: E402

obs = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
big = make_scene(num_frames=200, num_points=max(obs // 10, 1000), seed=5, run_max=18)
bp = ba.problem_from_map_frames(big, 198, 200, 2.0)
bs = ba.BundleAdjuster(device=0)
bs.load(bp)
bs.begin(default_solver_options())
bs.sweep(2)
bs.sync()
bs.set_timing(True)
bs.sweep(reps)
bs.sync()
kt = bs.kernel_times()["linearize"]
wb = bs.kernel_work()["linearize"][0]
print("obs %d points %d: %.1f us per launch, %.0f GB/s" % (bp.num_obs, bp.num_points, 1e3 * kt[0],
                                                           wb / (kt[0] * 1e-3) / 1e9), flush=True)
bs.close()
