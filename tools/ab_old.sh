#!/bin/bash
# Same-box comparison with another tree (e.g. a previous round's, built under ab_old/):
#   tools/ab_old.sh <rounds> <old_dir>
R=${1:-2}; OLD=${2:-ab_old}
for i in $(seq 1 $R); do
  timeout -k 10 200 python bench.py --steps 5 --warmup 5 --no-cpu --no-extras 2>/dev/null | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('new', round(b['value']/1e6,2))" || exit 1
  (cd $OLD && timeout -k 10 200 python bench.py --steps 5 --warmup 5 --no-cpu 2>/dev/null) | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('old', round(b['value']/1e6,2))" || exit 1
done
