#!/bin/bash
# Dissected-band Cholesky A/B: BA parity tests (split on), then the bench with the split on and off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ab}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  tests/test_ba_gpu.py tests/test_multirank_local_gpu.py tests/test_incremental_gpu.py > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-runs 0 --cpu-seconds 0 --frontend 0 > gpurun_out/bench_${TAG}_split.json 2> gpurun_out/bench_${TAG}_split.err || exit $?
SG_CHOL_SPLIT=0 timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-runs 0 --cpu-seconds 0 --frontend 0 > gpurun_out/bench_${TAG}_nosplit.json 2> gpurun_out/bench_${TAG}_nosplit.err || exit $?
python - <<PY
import json
for v in ("split", "nosplit"):
    d = json.load(open("gpurun_out/bench_${TAG}_%s.json" % v))
    o = d.get("other_workload", {})
    print(v, "C2 %.1f it/s chol %.2f us | C5 %.1f it/s chol %.2f us" % (d["value"], d["roofline"]["us_per_launch"],
          o.get("value", 0), o.get("roofline", {}).get("us_per_launch", 0)))
PY
