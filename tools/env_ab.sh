#!/bin/bash
# A/B of environment switches on the default library: for each "NAME=VALUE[,NAME=VALUE]" spec (or "base"), the
# C2 and C5 bench lines alone, printed as iterations/s and per-kernel us per iteration.
# Usage: env_ab.sh <tag> <spec> [<spec> ...]
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}; shift
for spec in "$@"; do
  envs=()
  [ "$spec" != "base" ] && IFS=',' read -ra envs <<< "$spec"
  n=$(echo "$spec" | tr '=,' '_-')
  for w in C2 C5; do
    st=20; [ $w = C2 ] && st=50
    env "${envs[@]}" timeout -k 10 200 python bench.py --only $w --steps $st --warmup 5 \
      > gpurun_out/envab_${TAG}_${n}_$w.json 2>gpurun_out/envab_${TAG}_${n}_$w.err || { echo "$spec $w failed"; tail -3 gpurun_out/envab_${TAG}_${n}_$w.err; exit 1; }
  done
  python - "$TAG" "$n" "$spec" <<'PY'
import json, sys
t, n, spec = sys.argv[1:4]
for w in ("C2", "C5"):
    d = json.loads(open("gpurun_out/envab_%s_%s_%s.json" % (t, n, w)).read().strip().splitlines()[-1])
    print(spec, w, round(d["value"], 1), {k: round(v * 1e3, 1) for k, v in d["kernel_ms_per_iter"].items() if v})
PY
done
