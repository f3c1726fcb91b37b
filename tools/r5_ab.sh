#!/bin/bash
# GPU tests (-x), then env A/B lines (tools/env_ab.sh) and the scaled sweep alone.  Usage: r5_ab.sh <tag> <spec>...
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
bash tools/env_ab.sh "$TAG" "$@" || exit 1
for spec in "$@"; do
  envs=(); [ "$spec" != "base" ] && IFS=',' read -ra envs <<< "$spec"
  env "${envs[@]}" timeout -k 10 200 python bench.py --only sweep --steps 20 --warmup 5 > gpurun_out/sweep_${TAG}_$(echo $spec | tr '=,' '_-').json 2>/dev/null || { echo "sweep $spec failed"; exit 1; }
  python - gpurun_out/sweep_${TAG}_$(echo $spec | tr '=,' '_-').json "$spec" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["result"]
u = d["update_lin"]
print(sys.argv[2], "sweep k_linearize %.1f us frac %.3f | k_update_lin %.1f us frac %.3f" % (d["ms_per_launch"] * 1e3, d["frac"], u["ms_per_launch"] * 1e3, u["frac"]))
PY
done
