# Full GPU round: tests, smoke, sweep, bench, rocprofv3 kernel trace + PMC passes
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 180 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
if [ "${SWEEP:-0}" = 1 ]; then
timeout -k 10 200 python tools/sweep.py --tree t125 --rounds 15 --out gpurun_out/sweep_t125.json > gpurun_out/sweep.txt 2>&1 || { echo sweep failed; tail gpurun_out/sweep.txt; exit 1; }
cat gpurun_out/sweep.txt
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --only-headline --no-b2b > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo prof failed; tail -20 $R/gpurun_out/prof_bench.err; exit 1; }
bash $R/tools/gpu_pmc.sh t125 > $R/gpurun_out/pmc.txt 2>&1 || { echo pmc failed; tail $R/gpurun_out/pmc.txt; exit 1; }
echo "done $(date)"
