#!/bin/bash
# config 4 on the 7-server pool: section profile (HP21 = -DMR_PROF variant) and PMC passes of the
# product library (divergence, LDS, traffic). usage: bash tools/r06_c4_evidence.sh <tag>
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; mkdir -p $O
MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/HP21.so timeout -k 10 300 python tools/prof.py snapshot_install_unreliable_2d 262144 7 > $O/prof_c4.txt 2>&1 || { echo "PROF FAIL"; tail $O/prof_c4.txt; exit 1; }
tail -8 $O/prof_c4.txt
bash tools/pmc.sh $O/pmc --test snapshot_install_unreliable_2d --nodes 7 --clusters 262144 --no-safety --variant= --million 0 --steps 1 --warmup 0 --pipeline 1 || { echo "pmc FAILED"; exit 1; }
python tools/pmc_sum.py $O/pmc --json $O/pmc_c4.json --test snapshot_install_unreliable_2d --clusters 262144 > $O/pmc_c4_summary.txt 2>&1; tail -8 $O/pmc_c4_summary.txt
