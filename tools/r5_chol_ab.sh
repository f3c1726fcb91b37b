#!/bin/bash
# Timing-only Cholesky A/B: phase traces of variant libraries (tools/build_variant.sh) beside the default.
# Usage: tools/r5_chol_ab.sh TAG name1 name2 ...   (libslamgpu_<name>.so; "base" = the default library)
set -o pipefail
tag=${1:?tag}; shift
out=gpurun_out/chol_ab_$tag.log
mkdir -p gpurun_out
: > $out
for v in "$@"; do
  for c in C2 C5; do
    echo "=== $v $c" >> $out
    if [ "$v" = base ]; then lib=""; else lib=slam-robot_amd/csrc/libslamgpu_$v.so; fi
    SG_LIB_PATH=$lib timeout -k 10 120 python3 -u tools/phase_trace.py $c >> $out 2>&1 || exit $?
  done
done
grep -E '^===|sum|phase 9|config' $out || true
