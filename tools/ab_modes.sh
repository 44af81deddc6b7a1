#!/bin/bash
# Interleaved same-box A/B of engine libraries in three regimes: the headline ensemble (open loop),
# one simulation alone open loop, one simulation alone closed loop.
#   tools/ab_modes.sh ROUNDS NAME...  (NAME "main" = libprimeuncore.so, else libprimeuncore_NAME.so)
R=$1; shift
for i in $(seq 1 $R); do
  for mode in ens single closed; do
    case $mode in
      ens) ARGS="--steps 5 --warmup 5 --no-cpu --no-extras";;
      single) ARGS="--replicas 1 --steps 3 --warmup 5 --no-cpu --no-extras";;
      closed) ARGS="--replicas 1 --steps 3 --warmup 5 --no-cpu --no-extras --replay closed";;
    esac
    for v in "$@"; do
      if [ $v = main ]; then unset PRIMEUNCORE_LIB; else export PRIMEUNCORE_LIB=$PWD/primesim_amd/libprimeuncore_$v.so; fi
      timeout -k 10 200 python bench.py $ARGS 2>>gpurun_out/ab_modes.err | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$mode', '$v', round(b['value']) if b['value']<1e6 else round(b['value']/1e6,2))" || exit 1
    done
  done
done
