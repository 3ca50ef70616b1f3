# round-4: section profiles (MR_PROF) with the cooperative AppendEntries receive off / on
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof4
for v in P0 P1; do MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/$v.so timeout -k 10 300 python tools/prof.py figure_8_unreliable_2c 131072 > gpurun_out/prof4/prof_$v.txt 2>&1 || { echo "PROF FAIL $v"; tail gpurun_out/prof4/prof_$v.txt; exit 1; }; done
paste gpurun_out/prof4/prof_P0.txt gpurun_out/prof4/prof_P1.txt | cut -c1-150
