# round 4: the 15-client KV applier's batch prefetch (P1, MR_LIN15_PRE) vs per-entry loads (P0)
PTEST="linearizable" TESTS="persist_partition_unreliable_linearizable_3a snapshot_unreliable_recover_concurrent_partition_linearizable_3b" BARGS="--clusters 65536" bash tools/ab.sh ab7 P0 P1 || exit 1
