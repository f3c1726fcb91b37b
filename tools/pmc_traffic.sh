#!/bin/bash
# HBM traffic of the kernels bench.py prices (MI355X_MICROARCH.md HBM/rocprofv3 recipe): one rocprofv3
# --pmc pass per counter (FETCH_SIZE, WRITE_SIZE), kernel-filtered, over a short bench.py run; then
# tools/pmc_traffic.py turns the per-dispatch counters into profiles/<tag>_pmc_traffic.json.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r1}
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
KRE="k_chol_tiles|k_cholesky_window|k_linearize|k_schur|k_S_reduce|k_point_update|k_track_fb|k_hamming_slices"
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "$KRE" -d "$OUT/p$i" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 4 --cpu-seconds 0 > "$OUT/p$i.json" 2> "$OUT/p$i.log" \
    || { echo "pass $c failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_traffic.py" "$OUT" "$R/profiles/${TAG}_pmc_traffic.json"
