set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
echo "start $(date)"
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --extra-tree none > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo prof failed; tail -20 $R/gpurun_out/prof_bench.err; exit 1; }
echo "done $(date)"
