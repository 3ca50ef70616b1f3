# section profile of the headline kernel (-DMR_PROF variant HP): figure_8_unreliable_2c, 131072 clusters
mkdir -p gpurun_out/hprof
MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/HP.so timeout -k 10 300 python tools/prof.py figure_8_unreliable_2c 131072 > gpurun_out/hprof/prof16.txt 2>&1 || { echo "PROF FAIL"; tail gpurun_out/hprof/prof16.txt; exit 1; }
cat gpurun_out/hprof/prof16.txt
