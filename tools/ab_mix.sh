#!/bin/bash
# Interleaved same-box A/B of (library, environment) pairs on the bench headline or one simulation alone:
#   tools/ab_mix.sh ROUNDS multi|single NAME:LIB:ENV[,ENV]...   (LIB "main" = libprimeuncore.so, else
#   libprimeuncore_LIB.so; ENV "base" = none)
R=$1; MODE=$2; shift 2
if [ "$MODE" = single ]; then ARGS="--replicas 1 --steps 3 --warmup 5 --no-cpu --no-extras"; else ARGS="--steps 5 --warmup 5 --no-cpu --no-extras"; fi
for i in $(seq 1 $R); do
  for v in "$@"; do
    name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; envs=${rest#*:}
    ( if [ "$lib" != main ]; then export PRIMEUNCORE_LIB=$PWD/primesim_amd/libprimeuncore_$lib.so; fi
      [ "$envs" != "base" ] && for e in ${envs//,/ }; do export "$e"; done
      timeout -k 10 200 python bench.py $ARGS 2>>gpurun_out/ab_mix.err | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$name', round(b['value']) if b['value']<1e6 else round(b['value']/1e6,2))" ) || exit 1
  done
done
