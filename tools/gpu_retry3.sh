#!/bin/bash
# gpurun, retried ONLY when no box or slot was free (exit 3: nothing ran, nothing
# charged).  Any run that started is never retried.  Usage: tools/gpu_retry3.sh LOG TIMEOUT cmd...
LOG=$1; T=$2; shift 2
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  echo "[gpu_retry3] no free box (try $i), waiting" >> "$LOG.retries"
  sleep 120
done
echo "EXIT $rc" >> "$LOG"
exit $rc
