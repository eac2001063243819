# usage: gpurun --timeout 600 -- bash tools/gpu_xcd_stale.sh
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 120 python tools/xcd_stale.py 30 512 > gpurun_out/xcd_stale_1.txt 2>&1 || { tail -20 gpurun_out/xcd_stale_1.txt; exit 1; }
grep stale gpurun_out/xcd_stale_1.txt
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 tools/xcd_stale.py 30 512 > gpurun_out/xcd_stale_8.txt 2> gpurun_out/xcd_stale_8.err || { tail -20 gpurun_out/xcd_stale_8.err; exit 1; }
grep stale gpurun_out/xcd_stale_8.txt
