#!/bin/bash
# BA bench at several rounds-per-chunk settings (SG_LIN_MAXR) -- k_linearize / k_point_update granularity.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in ${MAXR_LIST:-1 2 4}; do
  echo -n "maxr=$r: "
  SG_LIN_MAXR=$r timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --frontend 0 --sweep-obs 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_iter']; print('value %.1f' % d['value'], {a: round(1e3*b,1) for a,b in k.items()})" || break
done
