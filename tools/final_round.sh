#!/bin/bash
# Round-end GPU session: all GPU tests, smoke, bench, rocprof kernel stats, then the PMC traffic passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-fin}
bash tools/gpu_round.sh $TAG || exit $?
timeout -k 10 700 bash tools/pmc_traffic.sh $TAG > gpurun_out/pmc_$TAG.log 2>&1 || { tail -5 gpurun_out/pmc_$TAG.log; exit 1; }
tail -3 gpurun_out/pmc_$TAG.log
