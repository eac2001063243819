# rocprofv3 kernel-trace stats of the bench headline (the reference's four calls, T125)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 3 --only-headline --no-b2b > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo bench prof failed; tail -20 $R/gpurun_out/prof_bench.err; exit 1; }
find $R/gpurun_out/prof -name "*kernel_stats.csv" | head -3
echo "prof done $(date)"
