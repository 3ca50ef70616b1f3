#!/bin/bash
# the GPU suite, then same-box A/B of the pool kernel's same-kind stay (ST) against the committed
# head (BASE). usage: bash tools/r05_ab_stay.sh <tag>
cd "$GRAFT_REPO_ROOT"
bash tools/r05_suite.sh ${1}_suite || exit 1
TESTS="figure_8_unreliable_2c figure_8_unreliable_crash" ROUNDS=2 bash tools/ab.sh ${1}_ab BASE ST
