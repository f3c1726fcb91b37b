"""Diagnostic: where the cycles of k_track_fb's Newton iteration go (SG_TRK_STAMP=1; BASELINE config 3:
640x480, 2000 tracks, 3 levels, 7x7).  Lane 0 of every wave accumulates s_memtime deltas per phase; printed
as cycles per Newton iteration (summed over waves / summed iterations), plus the kernel time per launch."""
import ctypes as C
import os
import sys

os.environ["SG_TRK_STAMP"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
from slamgpu.tracker import HessianTracker  # noqa: E402
from slamgpu.video import make_frames, seed_points  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 7
frames = make_frames(2)
pts = seed_points(2000)
t = HessianTracker(window=W, depth=3, device=0, retry_levels=0)
t.MakePyramid(frames[0], 0)
t.MakePyramid(frames[1], 1)
t.load_features(pts, pts)
t.run(0, 1, 2)
t.results()
buf = (C.c_ulonglong * 10)()
t.lib.sg_tracker_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
t.lib.sg_tracker_debug_stamps(t.h, buf, 10)   # (reset)
reps = 10
t.run(0, 1, reps)
out, acc, its = t.results()
ms, _ = t.kernel_ms()
t.lib.sg_tracker_debug_stamps(t.h, buf, 10)
names = ["stage check/load", "probe sampling", "sums 1 (ps, pq)", "score", "sums 2 + differences",
         "2x2 step + update", "template patch", "other"]
iters = buf[8]
print("W=%d: %d waves, %d Newton iterations over %d launches; %.3f ms per launch; longest track %d iterations"
      % (W, buf[9], iters, reps, ms / reps, int(its.max())))
tot = sum(buf[k] for k in range(8))
for k in range(8):
    print("  %-24s %8.0f cycles / iteration  (%4.1f %%)" % (names[k], buf[k] / max(iters, 1), 100.0 * buf[k] / max(tot, 1)))
print("  total %.0f cycles per Newton iteration (wave-summed); per launch %.3f us per iteration of the longest track"
      % (tot / max(iters, 1), ms / reps * 1e3 / max(int(its.max()), 1)))
