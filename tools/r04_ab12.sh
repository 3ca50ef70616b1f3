# round 4: Q1 (ab11 winner, MR_KV_REQ_BATCH) | PI + the pending slots' log indices read once per applier visit (MR_KV_PIDX); then section profiles of PI (PIP) and PI + the 15-client batch prefetch (PAP)
P=tests/test_gpu_parity.py
PIDS="$P::test_scenario_bit_exact[unreliable_3a] $P::test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a] $P::test_scenario_bit_exact[snapshot_unreliable_recover_concurrent_partition_linearizable_3b] $P::test_linearizable_kv_15_clients_7_servers $P::test_kv_unreliable_traced $P::test_linearizability_checker_bit_exact[unreliable_3a-256-200] $P::test_linearizability_checker_bit_exact[persist_partition_unreliable_linearizable_3a-512-100]" \
TESTS="unreliable_3a persist_partition_unreliable_linearizable_3a snapshot_unreliable_recover_concurrent_partition_linearizable_3b" BARGS="--clusters 65536" bash tools/ab.sh ab12 Q1 PI || exit 1
for v in PIP PAP; do
  MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/$v.so timeout -k 10 300 python tools/prof.py persist_partition_unreliable_linearizable_3a 65536 > gpurun_out/ab12/prof46_$v.txt 2>&1 || { echo "PROF FAIL $v"; exit 1; }
done
paste gpurun_out/ab12/prof46_PIP.txt gpurun_out/ab12/prof46_PAP.txt | cut -c1-170
