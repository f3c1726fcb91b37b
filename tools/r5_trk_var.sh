#!/bin/bash
# Tracker variant check: the bit-exact tracker tests and the C3 front-end bench on a variant library
# (tools/build_variant.sh).  Usage: tools/r5_trk_var.sh TAG name   ("base" = the default library)
set -o pipefail
tag=${1:?tag}; v=${2:?name}
mkdir -p gpurun_out
if [ "$v" = base ]; then lib=""; else lib=slam-robot_amd/csrc/libslamgpu_$v.so; fi
SG_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_tracker_gpu.py tests/test_tracker_modes.py tests/test_frontend.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_trkvar_${tag}_$v.log 2>&1 \
  || { echo "$v: tracker tests failed"; tail -20 gpurun_out/pytest_trkvar_${tag}_$v.log; exit 1; }
echo "$v: $(tail -1 gpurun_out/pytest_trkvar_${tag}_$v.log)"
bash tools/r5_trk_ab.sh $tag $v
