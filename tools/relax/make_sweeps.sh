#!/bin/bash
# Inputs of the GPU sweep measurement (tools/relax/sweep_bench.hip), on the CPU:
# C4 replica 0's bench stream (seed 4), run exactly for the bench's 204,800
# warm-up requests, then one relaxation sweep (sweep 2) of a window of W
# requests dumped for W = 1,024 and 4,096 into tools/relax/data/wW/.
set -e
cd "$(dirname "$0")"
g++ -O2 -std=c++17 -o relax_proto relax_proto.cpp
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o sweep_bench sweep_bench.hip
mkdir -p data
python3 dump_stream.py C4 4 4 250000 data/c4
for W in 1024 4096; do
  mkdir -p data/w$W
  RELAX_SKIP=204800 RELAX_DUMP=data/w$W RELAX_DUMP_SWEEP=2 ./relax_proto data/c4 1024 $W
done
rm -f data/c4.req data/c4.delay
