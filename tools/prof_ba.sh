#!/bin/bash
# rocprofv3 kernel-trace statistics of the BA bench (no CPU baseline, no front end).
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-p}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 10 --cpu-seconds 0 --frontend 0 --sweep-obs ${SWEEP_OBS:-0} > "$R/gpurun_out/bench_prof_$TAG.json" 2> "$R/gpurun_out/prof_$TAG.err" || { tail -20 "$R/gpurun_out/prof_$TAG.err"; exit 1; }
python3 - "$R/gpurun_out/prof_$TAG/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-60s n=%5s avg %8.1f us  min %8.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
PY
