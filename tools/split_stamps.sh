#!/bin/bash
# Per-phase Cholesky stamps: the working build with the dissected band on and off, and tools/variants/head.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ss}
L=slam-robot_amd/csrc/libslamgpu.so
cp $L /tmp/lib_cur.so
for cfg in C2 C5; do
  echo "== split $cfg";   timeout -k 10 200 python -u tools/tile_stamps.py $cfg || exit $?
  echo "== nosplit $cfg"; SG_CHOL_SPLIT=0 timeout -k 10 200 python -u tools/tile_stamps.py $cfg || exit $?
done > gpurun_out/stamps_$TAG.log 2>&1
cp tools/variants/head.so $L
for cfg in C2 C5; do
  echo "== head $cfg"; timeout -k 10 200 python -u tools/tile_stamps.py $cfg || { cp /tmp/lib_cur.so $L; exit 1; }
done >> gpurun_out/stamps_$TAG.log 2>&1
cp /tmp/lib_cur.so $L
grep -E "^==|total" gpurun_out/stamps_$TAG.log
