# Round 6 mid-round check on one box: the changed multi-process drop-in tests, the T125
# XCD-mapping A/B of the headline kernel, and one PMC pass of the T1.3B write-credit stalls.
# usage: gpurun --timeout 1200 -- bash tools/gpu_r06_check.sh
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06check
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_dropin_gpu.py -x -v --timeout 400 --timeout-method thread \
  -k "eight or two_peers_on_gpu or default_placement or slow_producer or adamw" > $O/dropin_subset.txt 2>&1
rc=$?
tail -15 $O/dropin_subset.txt
[ $rc -eq 0 ] || { echo "tests rc $rc"; exit $rc; }
timeout -k 10 150 python -u tools/store_order_ab.py --tree t125 --rounds 12 --launches 40 \
  --only xcd_b8,xcd_b16,xcd_b32 --out $O/store_order_t125_d.json > $O/store_order_t125_d.txt 2>&1 || exit 1
tail -2 $O/store_order_t125_d.txt | cut -c 1-300
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE \
  --output-format csv -d $O/pmc_credit -o run -- python3 $R/tools/kernel_driver.py t1.3b 3 > $O/pmc_credit.log 2>&1 || { tail -20 $O/pmc_credit.log; exit 1; }
find $O/pmc_credit -name "*counter_collection.csv" | head -3
