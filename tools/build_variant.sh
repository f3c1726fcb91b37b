#!/bin/bash
# Build an A/B variant of libslamgpu.so with extra defines for ba_solver.hip, into slam-robot_amd/csrc/
# libslamgpu_<name>.so (load it with SG_LIB_PATH=...).  Usage: build_variant.sh <name> <hipcc defines...>
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
C="$R/slam-robot_amd/csrc"
NAME=${1:?name}; shift
make -C "$C" -s
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I"$R/include" -I"$C" --offload-arch=gfx950 \
  -munsafe-fp-atomics "$@" -c "$C/ba_solver.hip" -o "$C/build/ba_solver_$NAME.o"
objs=$(ls "$C"/build/*.o | grep -v "ba_solver" | tr '\n' ' ')
/opt/rocm/bin/hipcc --offload-arch=gfx950 "$C/build/ba_solver_$NAME.o" $objs -shared -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib -o "$C/libslamgpu_$NAME.so"
echo "built $C/libslamgpu_$NAME.so"
