# Round-final record set on one box: -m gpu tests + smoke + the default bench line
# (gpu_check.sh), the rocprofv3 kernel-trace stats of the bench headline, and every hot-path
# kernel's rocprofv3 stats + FETCH/WRITE counter passes for T125 and T1.3B (gpu_kernels_all.sh)
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_check.sh || exit 1
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 3 --only-headline --no-b2b > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo bench prof failed; tail -20 $R/gpurun_out/prof_bench.err; exit 1; }
bash $R/tools/gpu_kernels_all.sh || exit 1
echo "final set done $(date)"
