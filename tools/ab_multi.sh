#!/bin/bash
# Interleaved same-box comparison of several engine builds on the bench headline:
#   tools/ab_multi.sh ROUNDS NAME... (NAME "main" = libprimeuncore.so, else libprimeuncore_NAME.so)
R=$1; shift
for i in $(seq 1 $R); do
  for v in "$@"; do
    if [ $v = main ]; then unset PRIMEUNCORE_LIB; else export PRIMEUNCORE_LIB=$PWD/primesim_amd/libprimeuncore_$v.so; fi
    timeout -k 10 200 python bench.py --steps 5 --warmup 5 --no-cpu --no-extras 2>>gpurun_out/ab_multi.err | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', round(b['value']/1e6,2))" || exit 1
  done
done
