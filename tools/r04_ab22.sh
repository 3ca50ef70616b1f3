# round 4: configs 2 and 4 (7 servers, 32-bit keys) under the per-key-width defaults: G0 HEAD | G1 four-slot rescan for
# 32-bit keys too | G2 no cooperative AppendEntries receive | G3 no four-slot rescan (64-bit keys)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab22; mkdir -p $O; V=$PWD/madraft_amd/lib/var
P=tests/test_gpu_parity.py
for f in G0 G1 G2 G3; do
  MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $P::test_snapshot_7_nodes $P::test_fail_agree_5_unreliable "$P::test_scenario_bit_exact[snapshot_install_unreliable_2d]" > $O/parity_$f.log 2>&1 || { echo "PARITY FAIL $f"; tail -15 $O/parity_$f.log; exit 1; }
  echo "$f parity: $(tail -1 $O/parity_$f.log)"
done
for r in 1 2; do
  for f in G0 G1 G2 G3; do
    MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 300 python tools/cfg_ab.py "$r $f" C2,C4 2>> $O/err.log | tee -a $O/summary.txt || { echo "CFG FAIL $f"; tail $O/err.log; exit 1; }
  done
done
