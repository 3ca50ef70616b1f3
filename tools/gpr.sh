#!/bin/bash
# gpurun with waiting for a free slot (exit 3 = no box/slot free: nothing ran, nothing charged)
# usage: gpr.sh <timeout_s> <logfile> <command>
to=$1; log=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "slot(s) on this pod are busy\|status=transient" $log; then echo "rc=$rc" >> $log; exit $rc; fi
  echo "try $i: no slot (rc=$rc), waiting" >> $log.tries
  sleep 150
done
exit 3
