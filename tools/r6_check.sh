#!/bin/bash
# Round 6 iteration check: the BA GPU tests (-x), then an A/B of library builds on C2 / C5 (tools/r6_ab.sh).
# Usage: r6_check.sh <tag> <test selection (-k expression or "all")> <workloads> <so>...
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}; shift
SEL=${1:?selection}; shift
if [ "$SEL" = all ]; then K=(); else K=(-k "$SEL"); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
WLS=${1:?workloads}; shift
bash tools/r6_ab.sh "$TAG" "$WLS" "$@"
