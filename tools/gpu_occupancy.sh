# occupancy / run-length microbenchmark (tools/occupancy.hip), T125 and T1.3B sizes, cold
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 180 ./build/occupancy ${1:-11} > gpurun_out/occupancy_t125.txt 2>&1 || { echo occupancy failed; cat gpurun_out/occupancy_t125.txt; exit 1; }
cat gpurun_out/occupancy_t125.txt
timeout -k 10 300 ./build/occupancy ${2:-5} t1.3b > gpurun_out/occupancy_t13b.txt 2>&1 || { echo occupancy t1.3b failed; cat gpurun_out/occupancy_t13b.txt; exit 1; }
cat gpurun_out/occupancy_t13b.txt
