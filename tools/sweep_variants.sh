#!/bin/bash
# Scaled-sweep timing of alternative builds (tools/variants/*.so) x rounds-per-chunk settings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
cp slam-robot_amd/csrc/libslamgpu.so /tmp/lib_orig.so
for v in tools/variants/*.so; do
  cp "$v" slam-robot_amd/csrc/libslamgpu.so
  for r in ${MAXR_LIST:-1 2 4 8}; do
    echo -n "$(basename $v) maxr=$r: "
    SG_LIN_MAXR=$r timeout -k 10 100 python tools/sweep_only.py ${SWEEP_OBS:-2000000} 10 || break 2
  done
done
cp /tmp/lib_orig.so slam-robot_amd/csrc/libslamgpu.so
