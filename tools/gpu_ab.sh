# Interleaved A/B of two library builds (tools/ab_build.sh) on one GPU box: kernel tests on b,
# then three a/b rounds of tools/tile_ab.py and tools/sweep.py on T125.
R=$GRAFT_REPO_ROOT; cd $R
DILOCO_HIP_LIB=$R/build_ab/lib_b.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "micro or tiny or ragged or t125 or tiled" > gpurun_out/pytest_ab.log 2>&1 || { echo pytest b failed; tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
for i in 1 2 3; do for v in a b; do
DILOCO_HIP_LIB=$R/build_ab/lib_$v.so timeout -k 10 120 python tools/tile_ab.py --tree t125 --tiles 0 --flags auto --rounds 7 --steps 10 2>/dev/null | grep -E "tile +0|fused" | sed "s/^/$v: /" || exit 1
DILOCO_HIP_LIB=$R/build_ab/lib_$v.so timeout -k 10 120 python tools/sweep.py --tree t125 --rounds 7 2>/dev/null | grep -E "flags=-1 grid=    0" | sed "s/^/$v: /" || exit 1
done; done
