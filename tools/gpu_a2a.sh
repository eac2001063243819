# exchange="a2a": kernel and emulated-replica parity, the one-rank RCCL transport test
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_a2a_gpu.py tests/test_rccl_gpu.py -x -v --timeout 170 --timeout-method thread > gpurun_out/pytest_a2a.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_a2a.log; exit 1; }
tail -3 gpurun_out/pytest_a2a.log
