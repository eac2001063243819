# usage: gpurun --timeout 600 -- bash tools/gpu_race_probe.sh
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 tools/xcd_stale.py 20 512 > gpurun_out/xcd_stale_8.txt 2> gpurun_out/xcd_stale_8.err || { tail -20 gpurun_out/xcd_stale_8.err; exit 1; }
grep stale gpurun_out/xcd_stale_8.txt
RACE_NB=25 RACE_M=67108864 RACE_ITERS=4 RACE_VARIANTS=slow_dl_copy_nt_bf16,dl_copy_nt_bf16,slow_dl_copy_bf16 bash tools/gpu_gloo_race.sh
