R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 120 ./build/mem_ceiling ${1:-15} > gpurun_out/mem_ceiling.txt 2>&1 || { echo mem_ceiling failed; cat gpurun_out/mem_ceiling.txt; exit 1; }
cat gpurun_out/mem_ceiling.txt
