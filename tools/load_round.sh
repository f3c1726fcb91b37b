#!/bin/bash
# Host-load GPU check: Hamming parity + bench leg, then the main.cpp replay with per-phase Load timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-l}
timeout -k 10 300 python -u -m pytest tests/test_hamming.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ham_$TAG.log 2>&1 && \
timeout -k 10 200 python -u -c "
import json, bench
print(json.dumps(bench.bench_hamming(0, 0)))" > gpurun_out/ham_$TAG.json 2> gpurun_out/ham_$TAG.err && \
SG_HOST_TIMING=1 timeout -k 10 300 python -u tools/e2e_replay.py gpurun_out/e2e_replay_$TAG.json > gpurun_out/e2e_replay_$TAG.log 2> gpurun_out/e2e_replay_$TAG.err
rc=$?
tail -2 gpurun_out/pytest_ham_$TAG.log; cat gpurun_out/ham_$TAG.json; cat gpurun_out/e2e_replay_$TAG.log; tail -4 gpurun_out/e2e_replay_$TAG.err
exit $rc
