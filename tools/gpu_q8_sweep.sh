# int8-wire kernels under every launch policy incl. AUTO (tools/cold_sweep.py --what q8), cold,
# both trees, after the int8 GPU tests
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_large_gpu.py tests/test_special_values_gpu.py -x -q --timeout 170 --timeout-method thread -k "int8 or q8" > gpurun_out/pytest_q8.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_q8.log; exit 1; }
tail -1 gpurun_out/pytest_q8.log
timeout -k 10 300 python tools/cold_sweep.py --tree t125 --rounds 15 --what q8 --out gpurun_out/q8_t125.json 2>/dev/null || exit 1
timeout -k 10 300 python tools/cold_sweep.py --tree t1.3b --rounds 7 --what q8 --out gpurun_out/q8_t13b.json 2>/dev/null || exit 1
