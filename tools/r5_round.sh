#!/bin/bash
# One GPU session of round 5: GPU tests, smoke, the driver's bench line, the main.cpp replay (host phases of
# every SolveFrames load), then the per-workload rocprofv3 evidence (tools/profile_round.sh).  Every GPU step
# has its own time limit and the chain stops at the first failure.  Usage: r5_round.sh <tag> [skip-profile]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${1:?tag}
# all GPU tests (no -x: an assertion failure still lets the measurements below run; a crash, a fault or the time
# limit stops the chain)
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
prc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu_$TAG.log | grep -v PASSED | head -20
tail -2 gpurun_out/pytest_gpu_$TAG.log
if [ $prc -ne 0 ] && [ $prc -ne 1 ]; then echo "pytest rc=$prc: stopping"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
  || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python - gpurun_out/bench_$TAG.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C2 %.1f it/s (%.4f ms), roofline frac %.5f, lm_regime %.1f it/s" % (d["value"], d["ms_per_step"], d["roofline"]["frac"], d["lm_regime"]["value"]))
print("kernels", d["kernel_ms_per_iter"])
print("cpu", d["cpu_baseline"] and d["cpu_baseline"]["value"], "model C2", (d.get("strong_scaling_model") or {}).get("speedup"))
o = d.get("other_workload") or {}
if o: print("C5 %.1f it/s kernels %s model %s" % (o["value"], o["kernel_ms_per_iter"], (o.get("strong_scaling_model") or {}).get("speedup")))
for k, v in (d.get("solve_all_frames") or {}).items():
    print("solve_all %s: %.1f it/s (%.3f ms), n %d, %s" % (k, v["iters_per_s"], v["ms_per_iter"], v["n"], v["cholesky"]))
PY
timeout -k 10 300 python tools/parity_pins.py > gpurun_out/parity_pins_$TAG.json 2> gpurun_out/parity_pins_$TAG.err \
  || { echo "parity pins failed"; tail -5 gpurun_out/parity_pins_$TAG.err; exit 1; }
SG_HOST_TIMING=1 timeout -k 10 300 python tools/e2e_replay.py gpurun_out/e2e_replay_$TAG.json > gpurun_out/e2e_$TAG.log 2> gpurun_out/e2e_phases_$TAG.log \
  || { echo "replay failed"; tail -20 gpurun_out/e2e_phases_$TAG.log; exit 1; }
tail -12 gpurun_out/e2e_$TAG.log
[ "$2" = "skip-profile" ] && exit 0
bash tools/profile_round.sh "$TAG" || exit 1
echo "round chain ok"
