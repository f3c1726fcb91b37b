#!/bin/bash
# Round-5 diagnostics: (1) MFMA-busy counters of k_schur / k_chol_tiles / k_update_lin at C5 and C2 (VERDICT r4
# Missing 3), (2) the main.cpp replay under a HIP-API + kernel + copy trace to find what delays the late queue
# starts.  Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}
OUT="$R/gpurun_out/diag_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for W in ${WLS:-C5 C2}; do
  echo "== $W mfma pmc"
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --kernel-include-regex "k_schur|k_chol_tiles|k_update_lin" -d "$OUT/mfma_$W" -o run --output-format csv \
    -- python3 "$R/bench.py" --only "$W" --steps 20 --warmup 5 --model-scaling 0 --weak 0 \
    > "$OUT/mfma_$W.json" 2> "$OUT/mfma_$W.log" || { echo "mfma pmc $W failed"; tail -5 "$OUT/mfma_$W.log"; exit 1; }
done
[ -n "$NO_TRACE" ] && exit 0
echo "== replay trace"
SG_HOST_TIMING=1 REPLAY_CONTROL_PASSES=1 timeout -k 10 500 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace \
  --output-format csv -d "$OUT/trace" -o run -- python3 "$R/tools/e2e_replay.py" "$OUT/e2e_trace.json" \
  > "$OUT/e2e.log" 2> "$OUT/e2e_phases.log" || { echo "replay trace failed"; tail -20 "$OUT/e2e_phases.log"; exit 1; }
tail -6 "$OUT/e2e.log"
for f in $(find "$OUT/trace" -name "*.csv"); do gzip -9 "$f"; done
du -sh "$OUT"
echo "diag ok"
