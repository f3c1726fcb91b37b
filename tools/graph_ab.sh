#!/bin/bash
# A/B of the hipGraph-captured LM iteration (SG_GRAPH): the BA tests with graphs on, then C2 and C5 bench lines
# with graphs off and on.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
SG_GRAPH=1 timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_incremental_gpu.py -x -q -m gpu \
  --timeout 200 --timeout-method thread > gpurun_out/pt_graph.log 2>&1
rc=$?; tail -2 gpurun_out/pt_graph.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 0 1; do
  SG_GRAPH=$v timeout -k 10 200 python bench.py --only C2 --steps 50 --warmup 10 > gpurun_out/g_c2_$v.json 2>/dev/null || exit 1
  SG_GRAPH=$v timeout -k 10 200 python bench.py --only C5 --steps 20 --warmup 5 > gpurun_out/g_c5_$v.json 2>/dev/null || exit 1
done
python - <<'PY'
import json
for c in ("c2", "c5"):
    for v in (0, 1):
        d = json.loads(open("gpurun_out/g_%s_%d.json" % (c, v)).read().strip().splitlines()[-1])
        print(c, "graph", v, round(d["value"], 1), "it/s", round(d["ms_per_step"], 4), "ms; lm_regime",
              round(d["lm_regime"]["value"], 1), "; from start", round(d["solve_from_start"]["iters_per_s_wall"], 1))
PY
