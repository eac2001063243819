# exploration: memory-system ceilings (microbench) + cold A/B of the product kernels
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 120 ./build/mem_ceiling 15 > gpurun_out/mem_ceiling.txt 2>&1 || { echo mem_ceiling failed; cat gpurun_out/mem_ceiling.txt; exit 1; }
cat gpurun_out/mem_ceiling.txt
timeout -k 10 240 python tools/cold_sweep.py --tree t125 --rounds 11 --what ${WHAT:-flags,tiles} --out gpurun_out/cold_sweep_t125.json > gpurun_out/cold_sweep_t125.txt 2>&1 || { echo sweep failed; tail -20 gpurun_out/cold_sweep_t125.txt; exit 1; }
cat gpurun_out/cold_sweep_t125.txt
