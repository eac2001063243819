# N = 8 rehearsal: eight gloo ranks on the one GPU, the bench's default
# arguments and deadline (the driver's N = 8 run uses RCCL over eight GPUs): every multi-rank
# leg the 8-GPU run will take -- T1.3B legs, a2a landing buffers, the bf16 codec error leg,
# the isolated child legs, the 8-process CPU baseline -- runs once before that run needs it.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
t0=$(date +%s)
DILOCO_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 \
  > gpurun_out/bench_n8_gloo.json 2> gpurun_out/bench_n8_gloo.err || { echo n8 rehearsal failed; tail -40 gpurun_out/bench_n8_gloo.err; exit 1; }
echo "wall $(( $(date +%s) - t0 )) s"
grep "done at\|skipping\|watchdog\|failed\|Error" gpurun_out/bench_n8_gloo.err | sort | uniq -c | head -60 || true
