# round 4: AppendEntries receive batches software-pipelined (AP1, MR_AE_PIPE: the next batch's loads before this batch's log writes) vs HEAD (AP0)
PTEST="test_scenario_bit_exact and (figure_8_unreliable_2c or figure_8_unreliable_crash or snapshot_install_unreliable_2d)" TESTS="figure_8_unreliable_2c figure_8_unreliable_crash snapshot_install_unreliable_2d" bash tools/ab.sh ab16 AP0 AP1 || exit 1
P=tests/test_gpu_parity.py
PIDS="$P::test_scenario_bit_exact[unreliable_3a] $P::test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a] $P::test_scenario_bit_exact[snapshot_unreliable_recover_concurrent_partition_linearizable_3b] $P::test_snapshot_7_nodes $P::test_kv_unreliable_traced" \
TESTS="unreliable_3a persist_partition_unreliable_linearizable_3a snapshot_unreliable_recover_concurrent_partition_linearizable_3b" BARGS="--clusters 65536" bash tools/ab.sh ab16k AP0 AP1 || exit 1
