# Interleaved cold A/B of two library builds (build_ab/lib_a.so, lib_b.so): kernel parity tests
# on b, then tools/cold_sweep.py (flags) on a, b, a, b, a, b
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
DILOCO_HIP_LIB=$R/build_ab/lib_b.so timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "micro or tiny or ragged or t125 or tiled or pack_sgd or fused" > gpurun_out/pytest_ab.log 2>&1 || { echo pytest b failed; tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
for i in 1 2 3; do for v in a b; do
DILOCO_HIP_LIB=$R/build_ab/lib_$v.so timeout -k 10 200 python tools/cold_sweep.py --tree t125 --rounds 9 --what flags --out gpurun_out/ab_${v}_$i.json 2>/dev/null | grep -E "nt_loads " | sed "s/^/$v: /" || exit 1
done; done
