#!/bin/bash
# Build an experiment variant of the engine library: tools/build_exp.sh NAME "-DFLAG ..."
# -> primesim_amd/libprimeuncore_NAME.so (host objects from the normal build)
set -e
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../primesim_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fwrapv -Wall -Wno-unused-function \
  -mllvm -amdgpu-sched-strategy=max-ilp $FLAGS -c -o ../../build/obj/engine_$NAME.o engine.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o ../libprimeuncore_$NAME.so ../../build/obj/engine_$NAME.o \
  ../../build/obj/uncore.o ../../build/obj/config.o ../../build/obj/stream.o ../../build/obj/msglog.o ../../build/obj/server.o \
  ../../build/obj/jit.o ../../build/obj/jit_src.o -L/opt/rocm/lib -lhiprtc -Wl,-rpath,/opt/rocm/lib
