#!/bin/bash
# gpurun client wrapper: retries only when the call never ran (status=transient:
# no box/slot, or the box was not provisioned); anything that ran is final.
# usage: tools/gpr.sh LOG TIMEOUT 'command'
LOG=$1; T=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG; then sleep 100; continue; fi
  exit $rc
done
exit $rc
