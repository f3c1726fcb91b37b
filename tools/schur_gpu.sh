#!/bin/bash
# Schur-kernel iteration: BA parity tests on the GPU, then the BA bench (C2 headline + C5) for a few segment
# counts (SG_SCHUR_SEGS) with per-kernel times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-s}
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py tests/test_multirank_local_gpu.py tests/test_incremental_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
for segs in ${SEGS:-768}; do
  SG_SCHUR_SEGS=$segs timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-runs 0 --cpu-seconds 0 --frontend 0 --sweep-obs 0 > gpurun_out/bench_${TAG}_$segs.json 2> gpurun_out/bench_${TAG}_$segs.err
  rc=$?
  [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_${TAG}_$segs.err; exit $rc; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}_$segs.json'))
o=d['other_workload']
print('segs $segs  C2 %.1f it/s  ms %.4f | C5 %.1f it/s ms %.4f' % (d['value'], d['ms_per_step'], o['value'], o['ms_per_step']))
print('  C2', d['kernel_ms_per_iter'])
print('  C5', o['kernel_ms_per_iter'])
"
done
exit 0
