#!/bin/bash
# Quick device check after a BA kernel change: the BA parity tests (single rank and in-process shards), then
# the C2 and C5 bench lines alone (kernel times per iteration) and k_schur's C5 stamps.  Usage: ab_c2c5.sh <tag>
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_multirank_local_gpu.py -x -q -m gpu \
  --timeout 200 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1
rc=$?
tail -2 gpurun_out/pt_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --only C2 --steps 50 --warmup 10 > gpurun_out/b_${TAG}_c2.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --only C5 --steps 20 --warmup 5 > gpurun_out/b_${TAG}_c5.json 2>/dev/null || exit 1
python - "$TAG" <<'PY'
import json, sys
for c in ("c2", "c5"):
    d = json.loads(open("gpurun_out/b_%s_%s.json" % (sys.argv[1], c)).read().strip().splitlines()[-1])
    print(c, round(d["value"], 1), {k: round(v * 1e3, 1) for k, v in d["kernel_ms_per_iter"].items()})
PY
[ -n "$SKIP_STAMPS" ] && exit 0
timeout -k 10 120 python tools/schur_stamps.py C5 > gpurun_out/schur_st_C5_$TAG.log 2>&1 && cat gpurun_out/schur_st_C5_$TAG.log
