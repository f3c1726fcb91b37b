#!/bin/bash
# k_schur variant A/B (round 5): each library x segment plan (equal points / SG_SEG_BAL=1), C2 and C5 bench lines
# alone.  Usage: r5_schur_ab.sh <tag> <so> [<so> ...]
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}; shift
for so in "$@"; do
  n=$(basename "$so" .so)
  for bal in 0 1; do
    for w in C2 C5; do
      st=20; [ $w = C2 ] && st=50
      if [ $bal = 1 ]; then export SG_SEG_BAL=1; else unset SG_SEG_BAL; fi
      SG_LIB_PATH="$R/$so" timeout -k 10 200 python bench.py --only $w --steps $st --warmup 5 \
        > gpurun_out/sab_${TAG}_${n}_${bal}_$w.json 2>/dev/null || { echo "$n $bal $w failed"; exit 1; }
    done
    unset SG_SEG_BAL
    python - "$TAG" "$n" "$bal" <<'PY'
import json, sys
t, n, bal = sys.argv[1:4]
out = []
for w in ("C2", "C5"):
    d = json.loads(open("gpurun_out/sab_%s_%s_%s_%s.json" % (t, n, bal, w)).read().strip().splitlines()[-1])
    k = d["kernel_ms_per_iter"]
    out.append("%s %.1f it/s schur %.1f us" % (w, d["value"], k["schur"] * 1e3))
print("%-16s bal=%s  %s" % (n, bal, " | ".join(out)))
PY
  done
done
