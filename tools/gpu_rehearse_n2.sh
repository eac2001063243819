# N = 2 rehearsal of bench.py's multi-rank path with two gloo ranks on the one GPU (RCCL refuses
# two ranks per device; the driver's multi-GPU runs use RCCL). EXTRA: extra bench arguments.
R=${GRAFT_REPO_ROOT:-.}
cd $R && mkdir -p gpurun_out
DILOCO_BENCH_BACKEND=gloo timeout -k 10 ${TO:-500} python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --detail gpurun_out/bench_detail_n2_gloo.json $EXTRA \
  > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { echo n2 rehearsal failed; tail -30 gpurun_out/bench_n2_gloo.err; exit 1; }
cat gpurun_out/bench_n2_gloo.json
wc -c gpurun_out/bench_n2_gloo.json
grep "done at\|skipping\|watchdog\|failed" gpurun_out/bench_n2_gloo.err || true
