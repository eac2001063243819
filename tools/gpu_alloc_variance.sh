# usage: gpurun --timeout 600 -- bash tools/gpu_alloc_variance.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/alloc_variance.py same fresh shift same > gpurun_out/alloc_variance.txt 2> gpurun_out/alloc_variance.err || { tail -20 gpurun_out/alloc_variance.err; exit 1; }
cat gpurun_out/alloc_variance.txt
