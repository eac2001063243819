# N = 8 rehearsal: eight gloo ranks on the one GPU (the driver's N = 8 run uses RCCL over eight
# GPUs), the bench's defaults (deadline included: the wall-time check). NP=4 rehearses N = 4. bench.py's own heartbeat
# names the running leg on stderr every 20 s. ARGS: extra bench arguments; TAG names the outputs.
R=${GRAFT_REPO_ROOT:-.}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-default}
NP=${NP:-8}
t0=$(date +%s)
DILOCO_BENCH_BACKEND=gloo timeout -k 10 ${LIMIT:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus $NP --detail gpurun_out/bench_detail_n${NP}_gloo_$TAG.json $ARGS \
  > gpurun_out/bench_n${NP}_gloo_$TAG.json 2> gpurun_out/bench_n${NP}_gloo_$TAG.err || { echo n$NP rehearsal failed; tail -40 gpurun_out/bench_n${NP}_gloo_$TAG.err; exit 1; }
echo "wall $(( $(date +%s) - t0 )) s"
cat gpurun_out/bench_n${NP}_gloo_$TAG.json
wc -c gpurun_out/bench_n${NP}_gloo_$TAG.json
grep "done at\|skipping\|watchdog\|failed\|Error" gpurun_out/bench_n${NP}_gloo_$TAG.err | sort -u | head -60 || true
