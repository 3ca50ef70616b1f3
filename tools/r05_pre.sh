#!/bin/bash
# A/B of the early-loaded applier entries: kvraft (BASEK vs PRE) and the pool kernel (BASE vs PRE2)
cd "$GRAFT_REPO_ROOT"
NOPMC=1 bash tools/r05_kvab.sh ${1}_kv BASEK PRE || exit 1
PTEST="figure_8_unreliable_2c or figure_8_unreliable_crash or fail_agree_2b" TESTS="figure_8_unreliable_2c figure_8_unreliable_crash" ROUNDS=2 bash tools/ab.sh ${1}_pool BASE PRE2
