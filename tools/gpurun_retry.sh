#!/bin/bash
# gpurun with queueing: retry only while the pool reports no free box/slot (exit 3, nothing
# ran, nothing charged); any other outcome is final.  usage: tools/gpurun_retry.sh <timeout> <cmd...>
t=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $t -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[retry] no box free, waiting 120 s ($i)"
  sleep 120
done
exit 3
