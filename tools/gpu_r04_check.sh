# Round-4 GPU check: the drop-in / RCCL / mirror tests touched this round, then the bench line.
# usage: gpurun --timeout 1200 -- bash tools/gpu_r04_check.sh [pytest -k expr]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 780 python -u -m pytest tests/test_rccl_gpu.py tests/test_dropin_gpu.py \
  tests/test_train_loop_gpu.py tests/test_configs_gpu.py -m gpu -x -v --timeout 400 \
  --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_r04.log 2>&1 \
  || { echo "pytest failed"; tail -60 gpurun_out/pytest_r04.log; exit 1; }
tail -3 gpurun_out/pytest_r04.log
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
  || { echo "bench failed"; tail -40 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
wc -c gpurun_out/bench.json
