#!/bin/bash
# dev: tools/cfg_ab.py over variant libraries (two alternating rounds); CFGS picks the configs
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; mkdir -p $O
V=$PWD/madraft_amd/lib/var
for r in 1 2; do
  for f in "$@"; do
    MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 300 python tools/cfg_ab.py $f ${CFGS:-C3,C3c} >> $O/cfg.txt 2>> $O/cfg.err || { echo "FAIL $f"; tail -5 $O/cfg.err; exit 1; }
  done
done
cat $O/cfg.txt
