#!/bin/bash
# Tracker GPU check: front-end parity tests, then the tracker bench leg (no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-t}
timeout -k 10 400 python -u -m pytest tests/test_tracker_gpu.py tests/test_tracker_modes.py tests/test_frontend.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_trk_$TAG.log 2>&1 && \
timeout -k 10 200 python -u -c "
import json, bench
print(json.dumps(bench.bench_tracker(0, 0)))" > gpurun_out/trk_$TAG.json 2> gpurun_out/trk_$TAG.err
rc=$?
tail -3 gpurun_out/pytest_trk_$TAG.log; cat gpurun_out/trk_$TAG.json; tail -3 gpurun_out/trk_$TAG.err
exit $rc
