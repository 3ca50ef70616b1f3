#!/bin/bash
# section profile (-DMR_PROF variant HP, tools/var.py) of the headline, pool kernel and step kernel
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r05prof}; mkdir -p $O
for p in 1 0; do
  for n in ${SIZES:-8192 131072}; do
    echo "== pool=$p clusters=$n"
    MR_POOL=$p MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/HP.so timeout -k 10 120 python tools/prof.py ${TEST:-figure_8_unreliable_2c} $n > $O/prof_pool${p}_$n.txt 2>&1 || { echo "PROF FAIL"; tail $O/prof_pool${p}_$n.txt; exit 1; }
    cat $O/prof_pool${p}_$n.txt
  done
done
