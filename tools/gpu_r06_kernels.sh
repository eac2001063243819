# Round 6: the kernel-level GPU tests after the XCD-run mapping of dl_delta_pack_sgd, and the
# interleaved A/B of the product kernel against the round-5 mapping (xcd_b1) at both sizes.
# usage: gpurun --timeout 900 -- bash tools/gpu_r06_kernels.sh
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06kern
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_special_values_gpu.py -x -q \
  --timeout 300 --timeout-method thread > $O/kernel_tests.txt 2>&1
rc=$?
tail -4 $O/kernel_tests.txt
[ $rc -eq 0 ] || { echo "tests rc $rc"; exit $rc; }
timeout -k 10 120 python -u tools/store_order_ab.py --tree t125 --rounds 12 --launches 40 \
  --only xcd_b1,xcd_b16 --out $O/store_order_t125_e.json > $O/store_order_t125_e.txt 2>&1 || exit 1
timeout -k 10 150 python -u tools/store_order_ab.py --tree t1.3b --rounds 8 \
  --only xcd_b1,wire_first --out $O/store_order_t13b_e.json > $O/store_order_t13b_e.txt 2>&1 || exit 1
tail -1 $O/store_order_t125_e.txt | cut -c 1-400
tail -1 $O/store_order_t13b_e.txt | cut -c 1-400
