#!/bin/bash
# A/B of in-tree library builds (tools/build_variant.sh) on the C2 / C5 bench lines alone: iterations/s and the
# per-kernel us per iteration.  Usage: r6_ab.sh <tag> <workloads "C2 C5"> <so> [<so> ...]
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}; shift
WLS=${1:?workloads}; shift
for so in "$@"; do
  n=$(basename "$so" .so)
  for w in $WLS; do
    SG_LIB_PATH="$R/$so" timeout -k 10 200 python bench.py --only $w --steps 30 --warmup 5 \
      > gpurun_out/ab_${TAG}_${n}_$w.json 2>gpurun_out/ab_${TAG}_${n}_$w.log || { echo "$n $w failed"; tail -3 gpurun_out/ab_${TAG}_${n}_$w.log; exit 1; }
    python - "$TAG" "$n" "$w" <<'PY'
import json, sys
t, n, w = sys.argv[1:4]
d = json.loads(open("gpurun_out/ab_%s_%s_%s.json" % (t, n, w)).read().strip().splitlines()[-1])
print(n, w, round(d["value"], 1), {k: round(v * 1e3, 1) for k, v in d["kernel_ms_per_iter"].items()}, flush=True)
PY
  done
done
