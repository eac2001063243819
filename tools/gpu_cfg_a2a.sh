# the 1.3B config tests (tests/test_configs_gpu.py), all five in one process
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -x -v --timeout 500 --timeout-method thread > gpurun_out/pytest_cfg.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_cfg.log; exit 1; }
tail -3 gpurun_out/pytest_cfg.log
