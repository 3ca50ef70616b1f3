#!/bin/bash
# one gpurun call; when no box or slot is free (exit 3: nothing ran, nothing charged) wait and
# ask again, at most 6 times. Any other outcome is final. usage: tools/gpu_call.sh <out> <timeout> <cmd>
out=$1; to=$2; shift 2
for i in 1 2 3 4 5 6; do
  timeout $((to + 1500)) /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 150
done
echo "EXIT $rc" >> $out
