set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
PYTHONFAULTHANDLER=1 timeout -k 10 300 python -u -m pytest tests/test_dropin_gpu.py -m gpu -x -v --timeout 90 --timeout-method thread -k "single_peer or host_writes or host_tensors or deepcopies" > gpurun_out/pytest_probe.log 2>&1; rc=$?
tail -80 gpurun_out/pytest_probe.log; exit $rc
