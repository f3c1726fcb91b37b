#!/bin/bash
# Cholesky diagnostics: per-phase owner chain (phase_trace.py) and per-wave stamp totals (tile_stamps.py), C2 / C5.
# Usage: tools/r5_chol.sh TAG   (outputs in gpurun_out/chol_TAG.log)
set -o pipefail
tag=${1:-r5_c}
out=gpurun_out/chol_$tag.log
mkdir -p gpurun_out
: > $out
for c in C2 C5; do
  timeout -k 10 120 python3 -u tools/phase_trace.py $c >> $out 2>&1 || exit $?
  timeout -k 10 120 python3 -u tools/tile_stamps.py $c >> $out 2>&1 || exit $?
done
cat $out
