#!/bin/bash
# Dissected-band balance at C2 only: stamps for bottom sizes 3, 4, 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
{ for nd in 3 4 5; do echo "== nd$nd C2"; SG_CHOL_ND=$nd timeout -k 10 200 python -u tools/tile_stamps.py C2 || exit $?; done; } > gpurun_out/stamps_ndc2.log 2>&1 || exit $?
grep -E "^==|total" gpurun_out/stamps_ndc2.log
