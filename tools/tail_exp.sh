#!/bin/bash
# dev: budget-split launches with dense resumption of the held clusters (MR_F_STREAM) vs one launch
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; mkdir -p $O; shift
for B in "$@"; do
  MR_STEP_BUDGET=$B timeout -k 10 300 python tools/stream.py 131072 0,s131072 >> $O/tail.txt 2>> $O/tail.err || { echo FAIL; tail $O/tail.err; exit 1; }
  echo "budget $B" >> $O/tail.txt
done
cat $O/tail.txt
