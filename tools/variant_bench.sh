#!/bin/bash
# Time alternative builds of libslamgpu.so (tools/variants/*.so) on the BA bench, one after the other.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
cp slam-robot_amd/csrc/libslamgpu.so /tmp/lib_orig.so
for v in tools/variants/*.so; do
  cp "$v" slam-robot_amd/csrc/libslamgpu.so
  echo -n "$(basename $v): "
  timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --sweep-obs 0 --frontend 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_iter']; print('value %.1f schur %.4f chol %.4f total %.4f' % (d['value'], k['schur'], k['cholesky'], d['ms_per_step']))" || break
done
cp /tmp/lib_orig.so slam-robot_amd/csrc/libslamgpu.so
