#!/bin/bash
# A/B of one environment switch on the C2 / C5 bench lines (same library): alternating runs with VAR=off / on.
# Usage: r6_env_ab.sh <tag> <workloads "C2 C5"> <VAR> <off value> <on value> [rounds]
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}; WLS=${2:?workloads}; VAR=${3:?var}; OFF=${4:?off}; ON=${5:?on}; N=${6:-2}
for r in $(seq 1 "$N"); do
  for val in "$OFF" "$ON"; do
    for w in $WLS; do
      env "$VAR=$val" timeout -k 10 200 python bench.py --only $w --steps 30 --warmup 5 \
        > gpurun_out/eab_${TAG}_${val}_${w}_$r.json 2>gpurun_out/eab_${TAG}_${val}_${w}_$r.log \
        || { echo "$VAR=$val $w failed"; tail -3 gpurun_out/eab_${TAG}_${val}_${w}_$r.log; exit 1; }
      python - "gpurun_out/eab_${TAG}_${val}_${w}_$r.json" "$VAR=$val" "$w" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], round(d["value"], 1), {k: round(v * 1e3, 1) for k, v in d["kernel_ms_per_iter"].items() if v}, flush=True)
PY
    done
  done
done
