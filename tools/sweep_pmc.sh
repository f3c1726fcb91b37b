#!/bin/bash
# PMC passes over the scaled sweep (one counter group per rocprofv3 run).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_linearize" -d "$R/gpurun_out/pmc/p$i" -o run --output-format csv -- python3 "$R/tools/sweep_only.py" ${SWEEP_OBS:-2000000} 5 > "$R/gpurun_out/pmc/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc/p$i.log"; exit 1; }
done
echo done
