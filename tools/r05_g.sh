#!/bin/bash
# PMC passes of the headline (stamped with the library hash) and the service pool's section profile
cd "$GRAFT_REPO_ROOT"; T=$1
PARTS="pmc" bash tools/r05_final.sh $T || exit 1
O=gpurun_out/$T; mkdir -p $O
for t in unreliable_3a snapshot_unreliable_recover_concurrent_partition_linearizable_3b; do
  MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/HPK.so timeout -k 10 300 python tools/prof.py $t 65536 > $O/prof_$t.txt 2>&1 || { echo "PROF FAIL $t"; tail $O/prof_$t.txt; exit 1; }
  cat $O/prof_$t.txt
done
