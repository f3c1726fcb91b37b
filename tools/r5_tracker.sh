#!/bin/bash
# Tracker GPU tests (bit-exact vs the oracle), the front-end bench alone and the Newton-loop stamps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}
timeout -k 10 400 python -u -m pytest tests/test_tracker_gpu.py tests/test_tracker_modes.py tests/test_frontend.py tests/test_corners.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_trk_$TAG.log 2>&1 \
  || { echo "tracker tests failed"; tail -30 gpurun_out/pytest_trk_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_trk_$TAG.log
timeout -k 10 200 python bench.py --only frontend --steps 20 --warmup 5 > gpurun_out/frontend_$TAG.json 2>/dev/null || { echo "frontend bench failed"; exit 1; }
python - gpurun_out/frontend_$TAG.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["result"]["tracker"]
print("tracker %.1f us/frame, %.3g tracks/s, longest %d its, %.2f us/it" % (d["ms_per_frame_tracking"] * 1e3, d["value"], d["newton_iterations_max_track"], d["us_per_newton_iteration_on_longest_track"]))
PY
timeout -k 10 200 python tools/tracker_stamps.py 7 > gpurun_out/tracker_stamps_$TAG.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/tracker_stamps_$TAG.log; exit 1; }
cat gpurun_out/tracker_stamps_$TAG.log
