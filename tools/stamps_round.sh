#!/bin/bash
# Diagnostic GPU session: per-phase cycle stamps of the tiled Cholesky (C2, C5) and the Schur kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-st}
timeout -k 10 120 python -u tools/tile_stamps.py C2 > gpurun_out/stamps_c2_$TAG.log 2>&1 && \
timeout -k 10 300 python -u tools/tile_stamps.py C5 > gpurun_out/stamps_c5_$TAG.log 2>&1
rc=$?
cat gpurun_out/stamps_c2_$TAG.log gpurun_out/stamps_c5_$TAG.log
exit $rc
