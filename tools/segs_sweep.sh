#!/bin/bash
# Schur segment count sweep (SG_SCHUR_SEGS) on the config-2 and config-5 BA bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for s in 256 384 512 768 1024; do
  SG_SCHUR_SEGS=$s timeout -k 10 200 python bench.py --steps 100 --warmup 10 --cpu-runs 0 --cpu-seconds 0 --frontend 0 > gpurun_out/segs_$s.json 2> gpurun_out/segs_$s.err || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/segs_$s.json')); k=d['kernel_ms_per_iter']; o=d['other_workload']
print('segs $s: C2 %.0f it/s schur %.4f S_reduce %.4f | C5 %.0f it/s schur %.4f S_reduce %.4f' % (d['value'], k['schur'], k['S_reduce'], o['value'], o['kernel_ms_per_iter']['schur'], o['kernel_ms_per_iter']['S_reduce']))"
done
