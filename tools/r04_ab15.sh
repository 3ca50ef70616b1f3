# round 4: kernel-argument laundering (each Dev field its own scalar value instead of one spilled
# 16-register tuple): LB0 HEAD | LN2 node events (MR_NE_LAUNDER + MR_LAUNDER_ALL) | LT LN2 + the tester (MR_T_LAUNDER)
PTEST="test_scenario_bit_exact and (figure_8_unreliable_2c or figure_8_unreliable_crash)" TESTS="figure_8_unreliable_2c figure_8_unreliable_crash" bash tools/ab.sh ab15 LB0 LN2 LT || exit 1
P=tests/test_gpu_parity.py
PIDS="$P::test_scenario_bit_exact[unreliable_3a] $P::test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a] $P::test_scenario_bit_exact[snapshot_unreliable_recover_concurrent_partition_linearizable_3b] $P::test_linearizable_kv_15_clients_7_servers $P::test_kv_unreliable_traced" \
TESTS="unreliable_3a persist_partition_unreliable_linearizable_3a snapshot_unreliable_recover_concurrent_partition_linearizable_3b" BARGS="--clusters 65536" bash tools/ab.sh ab15k LB0 LN2 LT || exit 1
