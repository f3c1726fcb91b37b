#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof kernel trace.  Every GPU step has its own time limit and
# the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.err")
rc=$?
echo "chain rc=$rc"
tail -3 gpurun_out/pytest_gpu_$TAG.log
cat gpurun_out/smoke_$TAG.log 2>/dev/null | tail -2
cat gpurun_out/bench_$TAG.json 2>/dev/null
exit $rc
