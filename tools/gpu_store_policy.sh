# store-policy microbenchmark (tools/store_policy.hip), T125 and T1.3B sizes, cold
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 120 ./build/store_policy ${1:-11} > gpurun_out/store_policy_t125.txt 2>&1 || { echo store_policy failed; cat gpurun_out/store_policy_t125.txt; exit 1; }
cat gpurun_out/store_policy_t125.txt
timeout -k 10 240 ./build/store_policy ${2:-5} t1.3b > gpurun_out/store_policy_t13b.txt 2>&1 || { echo store_policy t1.3b failed; cat gpurun_out/store_policy_t13b.txt; exit 1; }
cat gpurun_out/store_policy_t13b.txt
