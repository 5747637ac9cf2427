#!/bin/bash
# Submit one gpurun call, resubmitting only when no box/slot was available or
# the box failed while being prepared (exit 3 / "transient": nothing ran,
# nothing charged).  Any other outcome -- including a failing command -- ends
# here.  Usage: tools/gpurun_retry.sh TIMEOUT 'command'
# (TMV_RETRY_ATTEMPTS, default 20, attempts 150 s apart)
T=$1; shift
N=${TMV_RETRY_ATTEMPTS:-20}
for attempt in $(seq 1 "$N"); do
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
