#!/bin/bash
# Submit one gpurun call, resubmitting only when no box/slot was available or
# the box failed while being prepared (exit 3 / "transient": nothing ran,
# nothing charged).  Any other outcome -- including a failing command -- ends
# here.  Usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for attempt in 1 2 3 4 5 6 7 8; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  echo "$out" | tail -40
  if [ $rc -eq 3 ] || echo "$out" | grep -q "status=transient"; then
    echo "[retry] attempt $attempt: no box (rc=$rc); waiting 150 s"
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
