#!/bin/bash
# Interleaved same-box A/B of engine libraries on one simulation alone, open and closed loop:
#   tools/ab_multi_single.sh ROUNDS NAME...  (NAME "main" = libprimeuncore.so, else libprimeuncore_NAME.so)
R=$1; shift
for i in $(seq 1 $R); do
  for mode in single closed; do
    ARGS="--replicas 1 --steps 3 --warmup 5 --no-cpu --no-extras"; [ $mode = closed ] && ARGS="$ARGS --replay closed"
    for v in "$@"; do
      if [ $v = main ]; then unset PRIMEUNCORE_LIB; else export PRIMEUNCORE_LIB=$PWD/primesim_amd/libprimeuncore_$v.so; fi
      timeout -k 10 200 python bench.py $ARGS 2>>gpurun_out/ab_single.err | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$mode', '$v', round(b['value']))" || exit 1
    done
  done
done
