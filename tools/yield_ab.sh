#!/bin/bash
# Owner-yield A/B: stamps with the SIMD mate's MFMA yield on / off (C2, C5), BA tests, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-y}
{
for cfg in C2 C5; do
  echo "== yield $cfg";   timeout -k 10 200 python -u tools/tile_stamps.py $cfg || exit $?
  echo "== noyield $cfg"; SG_CHOL_YIELD=0 timeout -k 10 200 python -u tools/tile_stamps.py $cfg || exit $?
done
} > gpurun_out/stamps_$TAG.log 2>&1 || exit $?
grep -E "^==|total" gpurun_out/stamps_$TAG.log
bash tools/chol_round.sh ${TAG}b | tail -3
