#!/bin/bash
# Interleaved same-box A/B of environment variants of the bench (single replica or headline):
#   tools/ab_env.sh ROUNDS single|multi NAME=ENV[,ENV]... ("base" = no extra env)
R=$1; MODE=$2; shift 2
if [ "$MODE" = single ]; then ARGS="--replicas 1 --steps 3 --warmup 5 --no-cpu --no-extras"; else ARGS="--steps 5 --warmup 5 --no-cpu --no-extras"; fi
for i in $(seq 1 $R); do
  for v in "$@"; do
    name=${v%%=*}; envs=${v#*=}
    ( [ "$envs" != "base" ] && for e in ${envs//,/ }; do export "$e"; done
      timeout -k 10 200 python bench.py $ARGS 2>>gpurun_out/ab_env.err | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$name', round(b['value']) if b['value']<1e6 else round(b['value']/1e6,2), b['config'].get('engine_variant','')[:24])" ) || exit 1
  done
done
