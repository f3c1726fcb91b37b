#!/bin/bash
# Per-workload rocprofv3 evidence for bench.py's roofline fields (MI355X_MICROARCH.md HBM/rocprofv3 recipe):
# for each workload (C2, C5, the scaled sweep, the front end) one kernel-trace --stats run and two separate
# --pmc passes (FETCH_SIZE, WRITE_SIZE), and for C2 / C5 a third (the matrix-core counters, tools/pmc_mfma.py) of `bench.py --only <workload>` with the driver's arguments
# (--steps 20 --warmup 5), so every file holds that workload's own launches only:
#   profiles/<tag>_kernel_stats_<workload>.csv   rocprofv3 kernel statistics (the workload alone: no modelled shards)
#   profiles/<tag>_pmc_traffic_<workload>.json   HBM bytes per launch (tools/pmc_traffic.py)
# bench.py's traffic fields read the newest *_pmc_traffic_<workload>.json.  Usage: profile_round.sh <tag> [workloads]
# On a gpurun box only gpurun_out/ comes back: the summaries are written to gpurun_out/prof_<tag>/profiles/ as
# well; copy them into profiles/ after the call (cp gpurun_out/prof_<tag>/profiles/* profiles/).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}
WLS=${2:-"C2 C5 sweep frontend"}
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
KRE="k_chol_tiles|k_cholesky_window|k_linearize|k_cam_reduce|k_cam_finalize|k_schur|k_S_reduce|k_point_update|k_update_lin|k_upd_reduce|k_track_fb|k_find_matches|k_hamming_slices"
for W in $WLS; do
  echo "== $W kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_$W" -o run --output-format csv \
    -- python3 "$R/bench.py" --only "$W" --steps 20 --warmup 5 --model-scaling 0 --weak 0 > "$OUT/kt_$W.json" 2> "$OUT/kt_$W.log" \
    || { echo "kernel trace $W failed"; tail -5 "$OUT/kt_$W.log"; exit 1; }
  f=$(ls "$OUT"/kt_$W/run_kernel_stats.csv "$OUT"/kt_$W/*/run_kernel_stats.csv "$OUT"/kt_$W/*/*/run_kernel_stats.csv 2>/dev/null | head -1)
  mkdir -p "$OUT/profiles"
  [ -n "$f" ] && cp "$f" "$R/profiles/${TAG}_kernel_stats_${W}.csv" && cp "$f" "$OUT/profiles/${TAG}_kernel_stats_${W}.csv"
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    echo "== $W pmc $c"
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$KRE" -d "$OUT/pmc_$W/p$i" -o run \
      --output-format csv -- python3 "$R/bench.py" --only "$W" --steps 20 --warmup 5 --model-scaling 0 --weak 0 \
      > "$OUT/pmc_${W}_p$i.json" 2> "$OUT/pmc_${W}_p$i.log" \
      || { echo "pmc $c $W failed"; tail -5 "$OUT/pmc_${W}_p$i.log"; exit 1; }
  done
  python3 "$R/tools/pmc_traffic.py" "$OUT/pmc_$W" "$R/profiles/${TAG}_pmc_traffic_${W}.json" \
    "bench.py --only $W --steps 20 --warmup 5" || exit 1
  cp "$R/profiles/${TAG}_pmc_traffic_${W}.json" "$OUT/profiles/"
  if [ "$W" = C2 ] || [ "$W" = C5 ]; then
    echo "== $W pmc mfma"
    timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
      --kernel-include-regex "k_schur|k_chol_tiles" -d "$OUT/mfma_$W" -o run --output-format csv \
      -- python3 "$R/bench.py" --only "$W" --steps 20 --warmup 5 --model-scaling 0 --weak 0 \
      > "$OUT/mfma_$W.json" 2> "$OUT/mfma_$W.log" || { echo "pmc mfma $W failed"; tail -5 "$OUT/mfma_$W.log"; exit 1; }
    python3 "$R/tools/pmc_mfma.py" "$OUT/mfma_$W" "$R/profiles/${TAG}_pmc_mfma_${W}.json" \
      "bench.py --only $W --steps 20 --warmup 5" || exit 1
    cp "$R/profiles/${TAG}_pmc_mfma_${W}.json" "$OUT/profiles/"
  fi
done
