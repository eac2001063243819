# Write-through (sc1) stores vs plain / non-temporal: the store-policy microbenchmark, the
# bit-identity test of every store policy, then the product kernels' cold sweep (every policy
# interleaved in one process, tools/cold_sweep.py) on T125 and T1.3B, fp32 and int8 wires
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
bash tools/gpu_store_policy.sh 11 5 > /dev/null || exit 1
grep -E "check|fused|write4|copy" gpurun_out/store_policy_t125.txt
grep -E "fused|write4|copy" gpurun_out/store_policy_t13b.txt
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "store_policies or slotted" > gpurun_out/pytest_wt.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_wt.log; exit 1; }
tail -1 gpurun_out/pytest_wt.log
timeout -k 10 300 python tools/cold_sweep.py --tree t125 --rounds 11 --what flags,q8 --out gpurun_out/wt_sweep_t125.json 2>/dev/null || exit 1
timeout -k 10 400 python tools/cold_sweep.py --tree t1.3b --rounds 5 --what flags,q8 --out gpurun_out/wt_sweep_t13b.json 2>/dev/null || exit 1
