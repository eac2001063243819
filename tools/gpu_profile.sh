# Round profile set: rocprofv3 kernel-trace stats of the bench headline and of every hot-path
# kernel (tools/kernel_driver.py), then the FETCH/WRITE counter passes (tools/gpu_pmc.sh).
R=$GRAFT_REPO_ROOT
TREE=${1:-t125}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 3 --only-headline --no-b2b > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo bench prof failed; tail -20 $R/gpurun_out/prof_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kern -o run --output-format csv -- python3 $R/tools/kernel_driver.py $TREE 5 > $R/gpurun_out/prof_kern.log 2>&1 || { echo kernel prof failed; tail -20 $R/gpurun_out/prof_kern.log; exit 1; }
bash $R/tools/gpu_pmc.sh $TREE || exit 1
echo "profile done $(date)"
