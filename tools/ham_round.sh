#!/bin/bash
# Hamming-only GPU check: parity tests, then the matcher bench leg (no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-h}
timeout -k 10 300 python -u -m pytest tests/test_hamming.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ham_$TAG.log 2>&1 && \
timeout -k 10 200 python -u -c "
import json, bench
print(json.dumps(bench.bench_hamming(0, 0)))" > gpurun_out/ham_$TAG.json 2> gpurun_out/ham_$TAG.err
rc=$?
tail -2 gpurun_out/pytest_ham_$TAG.log; cat gpurun_out/ham_$TAG.json; tail -3 gpurun_out/ham_$TAG.err
exit $rc
