#!/bin/bash
# Cholesky iteration: BA parity tests, per-phase stamps at C2 and C5, the BA bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ch}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_ba_gpu.py tests/test_multirank_local_gpu.py tests/test_incremental_gpu.py > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_$TAG.log | head -20; exit $rc; }
{
for cfg in C2 C5; do echo "== $TAG $cfg"; timeout -k 10 200 python -u tools/tile_stamps.py $cfg || exit $?; done
} > gpurun_out/stamps_$TAG.log 2>&1 || exit $?
python tools/stamp_table.py gpurun_out/stamps_$TAG.log ${CMP:-}
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-runs 0 --cpu-seconds 0 --frontend 0 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit $?
python - <<PY
import json
d = json.load(open("gpurun_out/bench_${TAG}.json"))
o = d.get("other_workload", {})
print("C2 %.1f it/s chol %.2f us | C5 %.1f it/s chol %.2f us" % (d["value"], d["roofline"]["us_per_launch"],
      o.get("value", 0), o.get("roofline", {}).get("us_per_launch", 0)))
print(d["kernel_ms_per_iter"])
PY
