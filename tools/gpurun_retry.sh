#!/bin/bash
# gpurun, retried ONLY while no box/slot was available or the box failed while
# being prepared (nothing ran, nothing charged).  Any run that reached the GPU
# (pass or fail) is final.  usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$OUT"; then
    echo "[retry $i] $(grep -o 'status=[a-z]*' "$OUT" | head -1) rc=$rc" >> "$OUT.retries"
    sleep 60
    continue
  fi
  exit $rc
done
exit 3
