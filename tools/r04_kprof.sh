# section profiles of the kvraft kernels (-DMR_PROF variant KP): unreliable_3a, persist_partition_unreliable_linearizable_3a
mkdir -p gpurun_out/kprof
for t in unreliable_3a persist_partition_unreliable_linearizable_3a; do
  MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/KP.so timeout -k 10 300 python tools/prof.py $t 65536 > gpurun_out/kprof/$t.txt 2>&1 || { echo "PROF FAIL $t"; tail gpurun_out/kprof/$t.txt; exit 1; }
done
paste gpurun_out/kprof/unreliable_3a.txt gpurun_out/kprof/persist_partition_unreliable_linearizable_3a.txt | cut -c1-170
