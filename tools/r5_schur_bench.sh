#!/bin/bash
# tools/schur_bench.hip consumer-loop modes on heterogeneous (-1) and single-last-tile batches.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
for h in -1 4 5 3; do for m in 0 6 7 4; do
  timeout -k 5 60 ./tools/schur_bench_bin $m $h || exit 1
done; done > gpurun_out/schur_bench_modes_r5.log 2>&1
cat gpurun_out/schur_bench_modes_r5.log
