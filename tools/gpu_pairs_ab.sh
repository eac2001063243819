# dl_delta_pack / dl_gather with two chunks per workgroup (DL_TUNE_PAIRS):
# bit-identity tests, then the cold A/B interleaved in one process (tools/cold_sweep.py flags)
# on T125 and T1.3B, then the SQ wait / DRAM credit counters of both dl_delta_pack forms.
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out/pairs
# the pair walker is in the tuning build only (make -C diloco-swarm_amd/csrc TUNING=1)
export DILOCO_HIP_LIB=$R/diloco-swarm_amd/lib/libdiloco_hip_tuning.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "store_policies or ragged or micro or slot_rebound" > gpurun_out/pairs/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pairs/pytest.log; exit 1; }
tail -1 gpurun_out/pairs/pytest.log
timeout -k 10 300 python tools/cold_sweep.py --tree t125 --rounds 11 --what flags --out gpurun_out/pairs/sweep_t125.json > gpurun_out/pairs/sweep_t125.txt 2>&1 || { echo sweep t125 failed; tail gpurun_out/pairs/sweep_t125.txt; exit 1; }
grep -E "^(delta_pack|gather) " gpurun_out/pairs/sweep_t125.txt
timeout -k 10 400 python tools/cold_sweep.py --tree t1.3b --rounds 5 --what flags --out gpurun_out/pairs/sweep_t13b.json > gpurun_out/pairs/sweep_t13b.txt 2>&1 || { echo sweep t13b failed; tail gpurun_out/pairs/sweep_t13b.txt; exit 1; }
grep -E "^(delta_pack|gather) " gpurun_out/pairs/sweep_t13b.txt
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY" \
  "TCC_EA0_WRREQ_STALL TCC_TOO_MANY_EA_WRREQS_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_RDREQ_DRAM_CREDIT_STALL GRBM_GUI_ACTIVE GRBM_COUNT" \
  "TCC_HIT TCC_MISS TCC_TAG_STALL TCC_BUSY" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/pairs/p$i -o run -- python3 $R/tools/cold_driver.py t125 5 > $R/gpurun_out/pairs/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pairs/p$i.log; exit 1; }
done
python3 $R/tools/pmc_table.py $R/gpurun_out/pairs/counters_t125.json $(find $R/gpurun_out/pairs -name "*counter_collection.csv") > $R/gpurun_out/pairs/pmc_table.txt 2>&1 || { echo pmc_table failed; tail $R/gpurun_out/pairs/pmc_table.txt; exit 1; }
echo "pairs A/B done $(date)"
