# round-4: kvraft A/B (K0 = round-4 start, K1 = thread slots cluster-major + scenario-fixed config,
# K2 = K1 + cluster-major scalars), the cooperative AppendEntries receive's parity, PC sampling probe
PIDS="tests/test_gpu_parity.py::test_scenario_bit_exact[unreliable_3a] tests/test_gpu_parity.py::test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a]" PTEST="" TESTS="unreliable_3a persist_partition_unreliable_linearizable_3a" BARGS="--clusters 65536" bash tools/ab.sh ab3 K0 K1 K2 || exit 1
for v in AD2 AD1 AC; do MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "(test_scenario_bit_exact and figure_8_unreliable) or test_cooperative_append_receive" > gpurun_out/ab3/dbg_$v.log 2>&1; echo "$v: $(tail -1 gpurun_out/ab3/dbg_$v.log)"; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/ab3/list_avail.txt 2>&1; grep -i -A12 "pc.sampl\|PC Sampling" gpurun_out/ab3/list_avail.txt | head -40
