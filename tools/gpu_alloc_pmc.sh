# Counters per allocation instance of the headline kernel (tools/alloc_pmc.py), two passes.
# usage: gpurun --timeout 600 -- bash tools/gpu_alloc_pmc.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d $R/gpurun_out/apmc_tlb -o run --output-format csv -- python3 $R/tools/alloc_pmc.py 10 > $R/gpurun_out/apmc_tlb.json 2> $R/gpurun_out/apmc.err || { tail -20 $R/gpurun_out/apmc.err; exit 1; }
cat $R/gpurun_out/apmc_tlb.json
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/apmc_dram -o run --output-format csv -- python3 $R/tools/alloc_pmc.py 10 > $R/gpurun_out/apmc_dram.json 2>> $R/gpurun_out/apmc.err || { tail -20 $R/gpurun_out/apmc.err; exit 1; }
cat $R/gpurun_out/apmc_dram.json
ls -R $R/gpurun_out/apmc_tlb | head -20
