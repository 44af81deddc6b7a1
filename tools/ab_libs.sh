#!/bin/bash
# Interleaved same-box A/B/C... of engine libraries on the bench headline:
#   tools/ab_libs.sh <rounds> <lib>...   (paths; "main" = primesim_amd/libprimeuncore.so)
R=$1; shift
for i in $(seq 1 $R); do
  for L in "$@"; do
    if [ "$L" = main ]; then unset PRIMEUNCORE_LIB; else export PRIMEUNCORE_LIB=$PWD/$L; fi
    timeout -k 10 200 python bench.py --steps 5 --warmup 5 --no-cpu --no-extras 2>/dev/null | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L', round(b['value']/1e6,2), 'M/s')" || exit 1
  done
done
