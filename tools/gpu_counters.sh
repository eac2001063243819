# rocprofv3 counter passes on the cold driver (tools/cold_driver.py): memory-side stalls,
# request levels (latency), L2 hits, TA/TD/TCP busy and stall cycles, SQ waits, HBM bytes.
# One pass per run, each within the per-block counter limits (TCC 4, TA 2, TD 2, TCP 4,
# SQ 8, GRBM 2); summary by tools/pmc_table.py.
R=$GRAFT_REPO_ROOT
TREE=${1:-t125}
mkdir -p $R/gpurun_out/counters
cd /tmp && export TMPDIR=/tmp
i=0
for set in \
  "FETCH_SIZE" \
  "WRITE_SIZE" \
  "TCC_EA0_WRREQ_STALL TCC_TOO_MANY_EA_WRREQS_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_RDREQ_DRAM_CREDIT_STALL GRBM_GUI_ACTIVE GRBM_COUNT" \
  "TCC_EA0_RDREQ_LEVEL TCC_EA0_RDREQ TCC_EA0_WRREQ_LEVEL TCC_EA0_WRREQ" \
  "TCC_HIT TCC_MISS TCC_TAG_STALL TCC_BUSY" \
  "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TC_STALL TD_TD_BUSY TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
  "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY" ; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/counters/p$i -o run -- python3 $R/tools/cold_driver.py $TREE 5 > $R/gpurun_out/counters/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -5 $R/gpurun_out/counters/p$i.log; exit 1; }
  echo "pass $i done: $set"
done
python3 $R/tools/pmc_table.py $R/gpurun_out/counters_$TREE.json $(find $R/gpurun_out/counters -name "*counter_collection.csv")
