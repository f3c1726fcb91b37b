#!/bin/bash
# A/B of in-tree library builds (tools/build_variant.sh): for each .so, the C2, C5 and scaled-sweep bench lines
# alone, printed as iterations/s and per-kernel ms per iteration.  Usage: ab_libs.sh <tag> <so> [<so> ...]
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}; shift
for so in "$@"; do
  n=$(basename "$so" .so)
  for w in C2 C5 sweep; do
    st=20; [ $w = C2 ] && st=50
    SG_LIB_PATH="$R/$so" timeout -k 10 200 python bench.py --only $w --steps $st --warmup 5 \
      > gpurun_out/ab_${TAG}_${n}_$w.json 2>/dev/null || { echo "$n $w failed"; exit 1; }
  done
  python - "$TAG" "$n" <<'PY'
import json, sys
t, n = sys.argv[1], sys.argv[2]
for w in ("C2", "C5"):
    d = json.loads(open("gpurun_out/ab_%s_%s_%s.json" % (t, n, w)).read().strip().splitlines()[-1])
    print(n, w, round(d["value"], 1), {k: round(v * 1e3, 1) for k, v in d["kernel_ms_per_iter"].items()})
d = json.loads(open("gpurun_out/ab_%s_%s_sweep.json" % (t, n)).read().strip().splitlines()[-1])["result"]
print(n, "sweep", round(d["ms_per_launch"] * 1e3, 1), "us", round(d["frac"], 4))
PY
done
