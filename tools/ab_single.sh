#!/bin/bash
# single-replica (latency-mode) A/B: tools-style, prints accesses/s per lib
for i in 1 2; do
  for v in main ${AB_OTHER:-base}; do
    if [ $v = main ]; then unset PRIMEUNCORE_LIB; else export PRIMEUNCORE_LIB=$PWD/primesim_amd/libprimeuncore_$v.so; fi
    timeout -k 10 120 python bench.py --replicas 1 --steps 3 --warmup 5 --no-cpu --no-extras 2>>gpurun_out/ab_single.err | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', round(b['value']), 'accesses/s single replica')" || exit 1
  done
done
