#!/bin/bash
# same-box A/B of variant libraries (tools/ab.sh, pipeline 1: kernel times comparable), then the
# section profile of the HP (-DMR_PROF) variant on the headline. usage: bash tools/r06_ab_prof.sh <tag> <variants...>
cd "$GRAFT_REPO_ROOT"; T=$1; shift
TESTS="figure_8_unreliable_2c figure_8_unreliable_crash" ROUNDS=2 STEPS=5 BARGS="--pipeline 1" bash tools/ab.sh $T "$@" || exit 1
O=gpurun_out/$T; mkdir -p $O
MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/HP.so timeout -k 10 180 python tools/prof.py figure_8_unreliable_2c 131072 > $O/prof_pool.txt 2>&1 || { echo "PROF FAIL"; tail $O/prof_pool.txt; exit 1; }
cat $O/prof_pool.txt
