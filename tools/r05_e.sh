#!/bin/bash
# evidence part 1 (suite, smoke, bench, kernel trace), then the FAIR claim-rotation A/B
cd "$GRAFT_REPO_ROOT"
PARTS="suite bench" bash tools/r05_final.sh ${1} || exit 1
TESTS="figure_8_unreliable_2c figure_8_unreliable_crash" ROUNDS=2 bash tools/ab.sh ${1}_ab BASE FAIR
