#!/bin/bash
# gpurun with retries on infrastructure-side transients only (box lost while
# being prepared, back-off, no free slot).  A command that ran and failed is
# never retried.  Usage: tools/gpu.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpu_last.log 2>&1
  rc=$?
  if grep -q "status=transient\|backing off\|slot(s) on this pod are busy\|stopped responding while being prepared" /tmp/gpu_last.log \
     && ! grep -q "status=ok\|status=fail" /tmp/gpu_last.log; then
    echo "[gpu.sh] transient (try $i), waiting" >&2
    sleep 45
    continue
  fi
  tail -3 /tmp/gpu_last.log | cut -c1-400
  exit $rc
done
tail -3 /tmp/gpu_last.log | cut -c1-400
exit 3
