# FETCH/WRITE counter passes (tools/gpu_pmc.sh) for T125 and T1.3B
R=$GRAFT_REPO_ROOT
for TREE in t125 t1.3b; do
bash $R/tools/gpu_pmc.sh $TREE || exit 1
rm -rf $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
done
