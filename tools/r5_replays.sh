#!/bin/bash
# GPU tests, then the main.cpp replay (tools/e2e_replay.py) N times: how many loads start late per replay.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}
N=${2:-3}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 \
  || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
for i in $(seq 1 $N); do
  SG_HOST_TIMING=1 REPLAY_CONTROL_PASSES=1 timeout -k 10 300 python tools/e2e_replay.py gpurun_out/e2e_replay_${TAG}_$i.json \
    > gpurun_out/e2e_${TAG}_$i.log 2> gpurun_out/e2e_phases_${TAG}_$i.log || { echo "replay $i failed"; tail -20 gpurun_out/e2e_phases_${TAG}_$i.log; exit 1; }
  grep criteria gpurun_out/e2e_${TAG}_$i.log
done
echo "replays ok"
