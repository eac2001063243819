# resident-grid caps on the product kernels (tools/cold_sweep.py --what grids), cold
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/cold_sweep.py --tree t125 --rounds 21 --what grids --out gpurun_out/grids_t125.json 2>/dev/null || exit 1
timeout -k 10 400 python tools/cold_sweep.py --tree t1.3b --rounds 9 --what grids --out gpurun_out/grids_t13b.json 2>/dev/null || exit 1
