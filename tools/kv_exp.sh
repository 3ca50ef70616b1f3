#!/bin/bash
# dev: kvraft configs (C5, C5L) per variant library and lanes-per-wave setting
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; mkdir -p $O
V=$PWD/madraft_amd/lib/var
for f in "$@"; do
  for l in ${LPWS:-0 32}; do
    LPW=$l MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 300 python tools/cfg_ab.py "$f/lpw$l" ${CFGS:-C5,C5L} >> $O/kv.txt 2>> $O/kv.err || { echo "FAIL $f $l"; tail -5 $O/kv.err; exit 1; }
  done
done
cat $O/kv.txt
