# round 4: leader prev-term loads only where the append reads them (RW1 vs RW0), next[]/match[]
# only for a leader's event (PL = RW1 + that); same box
PTEST="(test_scenario_bit_exact and (figure_8_unreliable or fail_agree_2b)) or test_small_capacities or (test_safety_checks_bit_exact and figure_8_unreliable) or (test_apply_checker and figure_8_unreliable)" PMC=1 TESTS="figure_8_unreliable_2c figure_8_unreliable_crash" bash tools/ab.sh ab5 RW0 RW1 PL || exit 1
mkdir -p gpurun_out/ab5
MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/PK.so timeout -k 10 300 python tools/prof.py unreliable_3a 65536 > gpurun_out/ab5/prof_kv27.txt 2>&1 || { echo "PROF FAIL"; tail gpurun_out/ab5/prof_kv27.txt; exit 1; }
MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/PK.so timeout -k 10 300 python tools/prof.py persist_partition_unreliable_linearizable_3a 65536 > gpurun_out/ab5/prof_kv46.txt 2>&1 || { echo "PROF FAIL"; tail gpurun_out/ab5/prof_kv46.txt; exit 1; }
paste gpurun_out/ab5/prof_kv27.txt gpurun_out/ab5/prof_kv46.txt | cut -c1-160
