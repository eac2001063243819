# N = 8 rehearsal: eight gloo ranks on the one GPU (the driver's N = 8
# run uses RCCL over eight GPUs). Every multi-rank leg the 8-GPU run takes -- T1.3B legs, a2a
# landing buffers, the bf16 codec error leg, the 8-process CPU baseline -- runs before that
# run needs it. ARGS: extra bench arguments (default: the bench's defaults, deadline
# included: the wall-time check); TAG names the outputs.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${TAG:-default}
t0=$(date +%s)
# a long gloo leg logs nothing for minutes: a heartbeat file keeps gpurun's silence guard
# from taking the run for hung (the rank processes write their progress to the .err file)
( while sleep 45; do echo "$(( $(date +%s) - t0 )) s" >> gpurun_out/heartbeat_n8_$TAG.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
DILOCO_BENCH_BACKEND=gloo timeout -k 10 ${LIMIT:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 $ARGS \
  > gpurun_out/bench_n8_gloo_$TAG.json 2> gpurun_out/bench_n8_gloo_$TAG.err || { echo n8 rehearsal failed; tail -40 gpurun_out/bench_n8_gloo_$TAG.err; exit 1; }
echo "wall $(( $(date +%s) - t0 )) s"
grep "done at\|skipping\|watchdog\|failed\|Error" gpurun_out/bench_n8_gloo_$TAG.err | sort -u | head -80 || true
