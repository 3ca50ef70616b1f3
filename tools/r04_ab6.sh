# round 4: the 15-client KV apply's three words as one batch of loads (LB1) vs one per decision (LB0)
PTEST="linearizable" TESTS="persist_partition_unreliable_linearizable_3a snapshot_unreliable_recover_concurrent_partition_linearizable_3b" BARGS="--clusters 65536" bash tools/ab.sh ab6 LB0 LB1 || exit 1
