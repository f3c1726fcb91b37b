#!/bin/bash
# Dissected-band balance: Cholesky stamps at C2 for several bottom sizes, C5 default, then the BA bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-nd}
{
for nd in 3 4 5; do echo "== nd$nd C2"; SG_CHOL_ND=$nd timeout -k 10 200 python -u tools/tile_stamps.py C2 || exit $?; done
echo "== nosplit C2"; SG_CHOL_SPLIT=0 timeout -k 10 200 python -u tools/tile_stamps.py C2 || exit $?
for nd in 32 33 34; do echo "== nd$nd C5"; SG_CHOL_ND=$nd timeout -k 10 200 python -u tools/tile_stamps.py C5 || exit $?; done
} > gpurun_out/stamps_$TAG.log 2>&1 || exit $?
python tools/stamp_table.py gpurun_out/stamps_$TAG.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-runs 0 --cpu-seconds 0 --frontend 0 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit $?
python - <<PY
import json
d = json.load(open("gpurun_out/bench_${TAG}.json"))
o = d.get("other_workload", {})
print("C2 %.1f it/s chol %.2f us | C5 %.1f it/s chol %.2f us" % (d["value"], d["roofline"]["us_per_launch"],
      o.get("value", 0), o.get("roofline", {}).get("us_per_launch", 0)))
print(d["kernel_ms_per_iter"])
PY
