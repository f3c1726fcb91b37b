#!/bin/bash
# Kernel-time breakdown experiments for k_schur (SG_DBG switches; results are not valid solves).
for f in 0 1 2 4 3 7; do
  echo -n "SG_DBG=$f: "
  SG_DBG=$f timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --sweep-obs 0 --frontend 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_iter']; print('schur %.4f chol %.4f lin %.4f total %.4f' % (k['schur'], k['cholesky'], k['linearize'], d['ms_per_step']))"
done
