#!/bin/bash
# Cholesky phase-removal timing experiments (SG_DBG switches; results are not valid solves).
#   8: no trailing update   16: no W/z solve   32: no prefetch loads   64: no factor loop   128: no W stores
for f in 0 8 16 32 64 128 248; do
  echo -n "SG_DBG=$f: "
  SG_DBG=$f timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --sweep-obs 0 --frontend 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_iter']; print('schur %.4f chol %.4f total %.4f' % (k['schur'], k['cholesky'], d['ms_per_step']))"
done
