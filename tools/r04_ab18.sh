# round 4: LT1 the tester (body and threads) on the scenario-aware laundered argument copy too (MR_T_LAUNDER) vs LT0 (HEAD)
PTEST="test_scenario_bit_exact and (figure_8_unreliable_2c or figure_8_unreliable_crash or snapshot_install_unreliable_2d)" TESTS="figure_8_unreliable_2c figure_8_unreliable_crash snapshot_install_unreliable_2d" bash tools/ab.sh ab18 LT0 LT1 || exit 1
P=tests/test_gpu_parity.py
PIDS="$P::test_scenario_bit_exact[unreliable_3a] $P::test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a] $P::test_scenario_bit_exact[snapshot_unreliable_recover_concurrent_partition_linearizable_3b] $P::test_snapshot_7_nodes $P::test_kv_unreliable_traced" \
TESTS="unreliable_3a persist_partition_unreliable_linearizable_3a snapshot_unreliable_recover_concurrent_partition_linearizable_3b" BARGS="--clusters 65536" bash tools/ab.sh ab18k LT0 LT1 || exit 1
