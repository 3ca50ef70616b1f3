# round 4: LS1 the argument copy launders only the fields scenario S has (MR_LAUNDER_S, compile-time) vs LS0 (runtime null tests)
PTEST="test_scenario_bit_exact and (figure_8_unreliable_2c or figure_8_unreliable_crash or snapshot_install_unreliable_2d)" TESTS="figure_8_unreliable_2c figure_8_unreliable_crash snapshot_install_unreliable_2d" bash tools/ab.sh ab17 LS0 LS1 || exit 1
P=tests/test_gpu_parity.py
PIDS="$P::test_scenario_bit_exact[unreliable_3a] $P::test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a] $P::test_scenario_bit_exact[snapshot_unreliable_recover_concurrent_partition_linearizable_3b] $P::test_snapshot_7_nodes $P::test_kv_unreliable_traced" \
TESTS="unreliable_3a persist_partition_unreliable_linearizable_3a snapshot_unreliable_recover_concurrent_partition_linearizable_3b" BARGS="--clusters 65536" bash tools/ab.sh ab17k LS0 LS1 || exit 1
