#!/bin/bash
# Run one gpurun call, retrying only while gpurun reports a transient pool state (no free slot or box,
# a box lost while being prepared: exit 3, nothing ran, nothing charged).  Any other exit status ends it.  Usage: tools/gpurun_retry.sh LOG TIMEOUT 'COMMAND'
log=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  grep -q "status=transient" $log || exit $rc
  sleep 120
done
exit 3
