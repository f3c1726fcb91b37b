#!/bin/bash
# Round 6: where k_chol_tiles' phase time goes.  Three --pmc passes on the C2 workload alone
# (instruction fetch / cache, wait and issue cycles, LDS), each a run of its own, plus a kernel trace:
#   gpurun_out/r6_chol_pmc/pmc.json  per-launch counter means by kernel (tools/pmc_group.py)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
W=${1:-C2}
OUT="$R/gpurun_out/r6_chol_pmc_$W"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --only $W --steps 20 --warmup 5 --model-scaling 0 --weak 0"
KRE="k_chol_tiles|k_schur|k_update_lin"
P1="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P3="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_IFETCH_LEVEL SQ_INSTS_MFMA SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  echo "== pass $i: $P"
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$KRE" -d "$OUT/p$i" -o run --output-format csv \
    -- python3 $B > "$OUT/p$i.json" 2> "$OUT/p$i.log" || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_group.py" "$OUT/pmc.json" "$OUT/p1" "$OUT/p2" "$OUT/p3" || exit 1
echo "== kernel trace"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- python3 $B \
  > "$OUT/kt.json" 2> "$OUT/kt.log" || { echo "kernel trace failed"; tail -5 "$OUT/kt.log"; exit 1; }
echo done
