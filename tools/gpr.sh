#!/bin/bash
# gpurun with retries ONLY for infrastructure-side transients (nothing ran on a GPU in those cases)
# usage: gpr.sh LOGFILE TIMEOUT CMD
log=$1; to=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  if grep -q "status=transient\|stopped responding\|backing off\|slot(s) on this pod are busy" $log && ! grep -q "status=ok" $log; then
    sleep 60; continue
  fi
  break
done
tail -40 $log
