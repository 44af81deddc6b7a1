#!/bin/bash
# Interleaved same-box A/B of two engine builds on the bench headline:
#   tools/ab_bench.sh <rounds> [bench args...]
# A = primesim_amd/libprimeuncore.so, B = primesim_amd/libprimeuncore_exp.so
R=${1:-2}; shift
ARGS=${@:---steps 5 --warmup 5 --no-cpu --no-extras}
for i in $(seq 1 $R); do
  for v in A B; do
    if [ $v = B ]; then export PRIMEUNCORE_LIB=$PWD/primesim_amd/libprimeuncore_exp.so; else unset PRIMEUNCORE_LIB; fi
    timeout -k 10 200 python bench.py $ARGS 2>/dev/null | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', round(b['value']/1e6,2), 'M/s', 'halted', b['config']['halted_replicas'])" || exit 1
  done
done
