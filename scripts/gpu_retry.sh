#!/bin/bash
# Run one gpurun call; retry (after 150 s) only while nothing ran: the pool had
# no box (exit 3) or the box was lost before the command started (status
# "transient", nothing charged).  Never retries a command that ran.
out=$1; shift
rc=0
for i in $(seq 1 ${GPU_RETRIES:-30}); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ]; then echo "[retry $i: no box]" >> "$out.retries"; sleep 150; continue; fi
  if grep -q 'status=transient' "$out" && grep -qE 'charged=(0.0s|Nones)' "$out"; then
    echo "[retry $i: transient]" >> "$out.retries"; sleep 150; continue
  fi
  exit $rc
done
exit $rc
