# round-4: the cooperative AppendEntries receive on / off (MR_AE_COOP), same box
PTEST="(test_scenario_bit_exact and (figure_8_unreliable_2c or figure_8_unreliable_crash or linearizable_3a)) or test_cooperative_append_receive" PMC=1 TESTS="figure_8_unreliable_2c figure_8_unreliable_crash" bash tools/ab.sh ab4 AC0 AC || exit 1
TESTS="persist_partition_unreliable_linearizable_3a" NOPAR="AC0 AC" BARGS="--clusters 65536" bash tools/ab.sh ab4k AC0 AC || exit 1
