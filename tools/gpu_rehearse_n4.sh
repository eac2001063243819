# N = 4 rehearsal (four gloo ranks on the one GPU): the multi-rank legs incl. the two-stage one
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
DILOCO_BENCH_BACKEND=gloo timeout -k 10 ${TO:-500} python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 3 --warmup 1 ${ARGS:---extra-tree none --no-dropin} \
  > gpurun_out/bench_n4_gloo.json 2> gpurun_out/bench_n4_gloo.err || { echo n4 rehearsal failed; tail -30 gpurun_out/bench_n4_gloo.err; exit 1; }
grep "done at\|skipping\|watchdog\|failed" gpurun_out/bench_n4_gloo.err | sort | uniq -c | head -40 || true
