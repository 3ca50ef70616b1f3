#!/bin/bash
# A/B: pools that refill from the rest of a batch larger than the resident pools (AST) against
# chunks that each drain (CUR), on config 3's whole 1M job; parity of AST on the streaming tests
cd "$GRAFT_REPO_ROOT"; T=$1; O=gpurun_out/$T; mkdir -p $O; V=$PWD/madraft_amd/lib/var
MADRAFT_HIP_LIB=$V/AST.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "lanes_chunks or step_budget or (test_scenario_bit_exact and figure_8_unreliable)" > $O/parity_AST.log 2>&1 || { echo "PARITY FAIL"; tail -20 $O/parity_AST.log; exit 1; }
echo "AST parity: $(tail -1 $O/parity_AST.log)"
for r in 1 2; do
  for f in CUR AST; do
    MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 400 python tools/cfg_ab.py $f C3M,C3cM,C3 2>&1 | grep -v amdgpu.ids | tee -a $O/summary.txt || exit 1
  done
done
