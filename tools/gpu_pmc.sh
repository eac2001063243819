# rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE in separate runs) + kernel-trace stats
R=$GRAFT_REPO_ROOT
TREE=${1:-t125}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/tools/kernel_driver.py $TREE 5 > $R/gpurun_out/pmc_fetch.log 2>&1 || { echo fetch pass failed; tail -20 $R/gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/tools/kernel_driver.py $TREE 5 > $R/gpurun_out/pmc_write.log 2>&1 || { echo write pass failed; tail -20 $R/gpurun_out/pmc_write.log; exit 1; }
F=$(find $R/gpurun_out/pmc_fetch -name "*counter_collection.csv" | head -1)
W=$(find $R/gpurun_out/pmc_write -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_summary.py $F $W $TREE $R/gpurun_out/pmc_$TREE.json
