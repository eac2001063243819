# Round-4 profile set (one GPU call): rocprofv3 kernel-trace stats of the bench headline, the
# per-launch trace of the int8-wire kernels at T1.3B (tools/q8_spread.py),
# the FETCH / WRITE counter passes of every hot-path kernel (tools/gpu_pmc.sh), and the host
# cost of the four drop-in calls (tools/dropin_host_profile.py).
# usage: gpurun --timeout 1200 -- bash tools/gpu_r04_profile.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 3 --only-headline --detail $R/gpurun_out/prof_bench_detail.json > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo bench prof failed; tail -20 $R/gpurun_out/prof_bench.err; exit 1; }
cat $R/gpurun_out/prof_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_q8 -o run --output-format csv -- python3 $R/tools/q8_spread.py t1.3b 12 > $R/gpurun_out/q8_spread.json 2> $R/gpurun_out/q8_spread.err || { echo q8 prof failed; tail -20 $R/gpurun_out/q8_spread.err; exit 1; }
cat $R/gpurun_out/q8_spread.json
bash $R/tools/gpu_pmc.sh t125 || exit 1
cd $R && timeout -k 10 300 python3 tools/dropin_host_profile.py 300 > gpurun_out/dropin_host_profile.txt 2>&1 || { echo host profile failed; tail -20 gpurun_out/dropin_host_profile.txt; exit 1; }
head -12 gpurun_out/dropin_host_profile.txt
echo "profile done $(date)"
