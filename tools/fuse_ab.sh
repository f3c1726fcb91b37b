#!/bin/bash
# Fused-launch A/B: BA parity tests, then the BA bench with the fused launches on and off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-fu}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_ba_gpu.py tests/test_multirank_local_gpu.py tests/test_incremental_gpu.py > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_$TAG.log | head -20; exit $rc; }
for v in 1 0; do
  SG_FUSE=$v timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-runs 0 --cpu-seconds 0 --frontend 0 > gpurun_out/bench_${TAG}_$v.json 2> gpurun_out/bench_${TAG}_$v.err || exit $?
done
python - <<PY
import json
for v in ("1", "0"):
    d = json.load(open("gpurun_out/bench_${TAG}_%s.json" % v))
    o = d.get("other_workload", {})
    print("fuse", v, "C2 %.1f it/s %.4f ms | C5 %.1f it/s | from start %.1f it/s" % (d["value"], d["ms_per_step"], o.get("value", 0), d["solve_from_start"]["iters_per_s_wall"]))
    print("  ", d["kernel_ms_per_iter"])
PY
