# round 4: F1 the per-key-width defaults (four-slot rescan for 64-bit keys, cooperative AppendEntries receive for 32-bit keys) vs F0 (both off, HEAD 03bd586)
PTEST="test_scenario_bit_exact and (figure_8_unreliable_2c or figure_8_unreliable_crash or snapshot_install_unreliable_2d)" TESTS="figure_8_unreliable_2c figure_8_unreliable_crash snapshot_install_unreliable_2d" bash tools/ab.sh ab21 F0 F1 || exit 1
P=tests/test_gpu_parity.py
PIDS="$P::test_scenario_bit_exact[unreliable_3a] $P::test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a] $P::test_scenario_bit_exact[snapshot_unreliable_recover_concurrent_partition_linearizable_3b] $P::test_snapshot_7_nodes $P::test_cooperative_append_receive $P::test_linearizable_kv_15_clients_7_servers $P::test_kv_unreliable_traced" \
TESTS="unreliable_3a persist_partition_unreliable_linearizable_3a snapshot_unreliable_recover_concurrent_partition_linearizable_3b" BARGS="--clusters 65536" bash tools/ab.sh ab21k F0 F1 || exit 1
