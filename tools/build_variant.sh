#!/bin/bash
# Build an A/B variant of libslamgpu.so with extra defines for one kernel-family translation unit, into
# slam-robot_amd/csrc/libslamgpu_<name>.so (load it with SG_LIB_PATH=...).
# Usage: build_variant.sh <name> <tu: ba_sweep|ba_schur|ba_chol|ba_intr|ba_solver> <hipcc defines...>
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
C="$R/slam-robot_amd/csrc"
NAME=${1:?name}; shift
TU=${1:?translation unit}; shift
make -C "$C" -s
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I"$R/include" -I"$C" --offload-arch=gfx950 \
  -munsafe-fp-atomics "$@" -c "$C/$TU.hip" -o "$C/build/${TU}_$NAME.o.v"
objs=$(ls "$C"/build/*.o | grep -v "/$TU.o" | tr '\n' ' ')
/opt/rocm/bin/hipcc --offload-arch=gfx950 "$C/build/${TU}_$NAME.o.v" $objs -shared -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib -o "$C/libslamgpu_$NAME.so"
echo "built $C/libslamgpu_$NAME.so"
