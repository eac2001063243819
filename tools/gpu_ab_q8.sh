# int8-wire kernels: parity tests on b, then interleaved cold A/B of a and b (tools/cold_sweep.py q8)
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
DILOCO_HIP_LIB=$R/build_ab/lib_b.so timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_rccl_gpu.py -x -q --timeout 150 --timeout-method thread -k "int8 or q8" > gpurun_out/pytest_ab.log 2>&1 || { echo pytest b failed; tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
for i in 1 2 3; do for v in a b; do
DILOCO_HIP_LIB=$R/build_ab/lib_$v.so timeout -k 10 200 python tools/cold_sweep.py --tree ${TREE:-t125} --rounds 9 --what q8 --out gpurun_out/abq8_${TREE:-t125}_${v}_$i.json 2>/dev/null | sed "s/^/$v: /" || exit 1
done; done
