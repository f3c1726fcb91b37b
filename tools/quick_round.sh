#!/bin/bash
# Short GPU session: front-end GPU tests (Hamming, tracker), Cholesky stamps at C2/C5, and a bench without
# CPU legs.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -u -m pytest tests/test_hamming.py tests/test_ba_gpu.py tests/test_incremental_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_q_$TAG.log 2>&1 && \
timeout -k 10 120 python -u tools/tile_stamps.py C2 > gpurun_out/stamps_c2_$TAG.log 2>&1 && \
for dbg in 1 2 3; do echo "== SG_DBG=$dbg"; SG_DBG=$dbg timeout -k 10 120 python -u tools/tile_stamps.py C2 || exit 1; done > gpurun_out/stamps_c2_dbg_$TAG.log 2>&1 && \
timeout -k 10 300 python -u tools/tile_stamps.py C5 > gpurun_out/stamps_c5_$TAG.log 2>&1 && \
timeout -k 10 300 python -u tools/e2e_replay.py gpurun_out/e2e_replay_$TAG.json > gpurun_out/e2e_replay_$TAG.log 2>&1 && \
timeout -k 10 400 python -u bench.py --cpu-runs 0 --cpu-seconds 0 --sweep-obs 0 > gpurun_out/bench_q_$TAG.json 2> gpurun_out/bench_q_$TAG.err
rc=$?
tail -3 gpurun_out/pytest_q_$TAG.log
cat gpurun_out/stamps_c2_$TAG.log gpurun_out/stamps_c2_dbg_$TAG.log gpurun_out/stamps_c5_$TAG.log gpurun_out/e2e_replay_$TAG.log 2>/dev/null
exit $rc
