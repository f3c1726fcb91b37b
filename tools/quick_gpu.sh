#!/bin/bash
# Quick GPU iteration: BA parity tests, then the BA bench (no CPU baseline / front end) with kernel times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --frontend 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
python -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('value %.1f it/s  ms/step %.4f' % (d['value'], d['ms_per_step']))
print('kernels', d['kernel_ms_per_iter'])
print('sweep', d['roofline_sweep'])
print('sweep_scaled', d['roofline_sweep_scaled'])
" || tail -20 gpurun_out/bench_$TAG.err
exit $rc
