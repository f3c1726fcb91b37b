"""Profiling target: SolveAllFrames(C2 map, 2, solve_cameras) (main.cpp:327, slam.cpp:447-480): the whole map
with the intrinsics free, K always-linearize LM iterations.  Run under rocprofv3 --kernel-trace --stats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
from slamgpu import ba  # noqa: E402
from slamgpu.capi import default_solver_options  # noqa: E402
from slamgpu.scene import make_config  # noqa: E402

cams = len(sys.argv) < 2 or sys.argv[1] != "0"
m = make_config("C2")
p = ba.problem_from_map_all(m, 2.0, cams)
g = ba.BundleAdjuster()
g.load(p)
print(g.info())
g.begin(default_solver_options(max_num_iterations=100, disable_termination=1, always_linearize=1))
g.iterate(10)
g.sync()
print(g.summary())
