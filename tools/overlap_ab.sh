#!/bin/bash
# A/B of the Schur / camera-reduction overlap (SG_SCHUR_OVERLAP): C2 and C5 bench lines with it off and on.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 0 1; do  # SG_SCHUR_OVERLAP off / on
SG_SCHUR_OVERLAP=$v timeout -k 10 300 python bench.py --only C2 --steps 50 --warmup 10 > gpurun_out/ovl_c2_$v.json 2>/dev/null || exit 1
SG_SCHUR_OVERLAP=$v timeout -k 10 300 python bench.py --only C5 --steps 20 --warmup 5 > gpurun_out/ovl_c5_$v.json 2>/dev/null || exit 1
done
python - <<'PY'
import json
for c in ("c2","c5"):
    for v in (0,1):
        d=json.loads(open(f"gpurun_out/ovl_{c}_{v}.json").read().strip().splitlines()[-1])
        print(c, "overlap", v, round(d["value"],1), "it/s", {k: round(x*1e3,1) for k,x in d["kernel_ms_per_iter"].items()})
PY
