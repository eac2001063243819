# rocprofv3 kernel-trace stats of every hot-path kernel (tools/kernel_driver.py) and the
# FETCH/WRITE counter passes, for T125 and T1.3B
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for TREE in t125 t1.3b; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kern_$TREE -o run --output-format csv -- python3 $R/tools/kernel_driver.py $TREE 5 > $R/gpurun_out/prof_kern_$TREE.log 2>&1 || { echo kernel prof $TREE failed; tail -20 $R/gpurun_out/prof_kern_$TREE.log; exit 1; }
bash $R/tools/gpu_pmc.sh $TREE || exit 1
rm -rf $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
done
echo "kernels done $(date)"
