#!/bin/bash
# GPU session: BA GPU tests (incl. config 5), then the default bench (C2 headline + C5) with every leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-c5}
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
tail -3 gpurun_out/bench_$TAG.err
exit $rc
