R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dropin_gpu.py tests/test_train_loop_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/pytest_dropin.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_dropin.log; exit 1; }
tail -2 gpurun_out/pytest_dropin.log
timeout -k 10 450 python bench.py > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err || { echo bench failed; tail -30 gpurun_out/bench_h.err; exit 1; }
echo bench ok
