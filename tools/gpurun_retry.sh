#!/bin/bash
# Run one gpurun call, retrying only while the pool has no free slot (gpurun exit 3: nothing ran,
# nothing charged).  Any other exit status ends it.  Usage: tools/gpurun_retry.sh LOG TIMEOUT 'COMMAND'
log=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  grep -q "slot(s) on this pod are busy\|no free box\|no box" $log || exit $rc
  sleep 120
done
exit 3
