# every fp32 kernel's launch policy incl. write-through stores, interleaved cold, T125 (21 rounds)
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 400 python tools/cold_sweep.py --tree t125 --rounds 21 --what flags --out gpurun_out/wt_ab_t125.json 2>/dev/null | grep -E "nt_loads\+stores  |wt_stores|auto" || exit 1
