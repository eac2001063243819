# tools/alloc_history.py in three orders, each its own process, on one box.
# usage: gpurun --timeout 900 -- bash tools/gpu_alloc_history.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
for order in q8,q8,f32,q8 head,f32,head,q8,head f32,headdev,head,headdev; do
  timeout -k 10 240 python3 tools/alloc_history.py $order >> gpurun_out/alloc_history.txt 2>> gpurun_out/alloc_history.err || { tail -20 gpurun_out/alloc_history.err; exit 1; }
done
grep order gpurun_out/alloc_history.txt
