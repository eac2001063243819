# exchange="xgmi_inner": GPU tests (single replica, 2/4 processes), kernel profile, N = 2 rehearsal
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dropin_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "direct or peer_gather" > gpurun_out/pytest_xi.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_xi.log; exit 1; }
tail -2 gpurun_out/pytest_xi.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kern -o run --output-format csv -- python3 $R/tools/kernel_driver.py t125 5 > $R/gpurun_out/prof_kern.log 2>&1 || { echo kernel prof failed; tail -20 $R/gpurun_out/prof_kern.log; exit 1; }
cd $R && bash tools/gpu_rehearse_n2.sh > /dev/null && echo n2 ok
