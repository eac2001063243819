# Why the sharded fp32 exchange behind the calls runs slow with four gloo ranks on one GPU:
# bench's headline only at N = 2 and 4, a few steps each (same box, in turn). Answer
# (profiles/r05_gloo_n_probe.txt, tools/gloo_n_probe.py): gloo itself, when a reduce_scatter
# and an all_gather of device tensors are in flight together at four ranks.
R=${GRAFT_REPO_ROOT:-.}
cd $R && mkdir -p gpurun_out/n4probe
for np in 2 4; do
  DILOCO_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 2952$np bench.py --gpus $np \
    --only-headline --steps ${STEPS:-6} --warmup 1 --detail gpurun_out/n4probe/d_$np.json \
    > gpurun_out/n4probe/l_$np.json 2> gpurun_out/n4probe/e_$np.txt \
    || { echo "n=$np failed"; tail -20 gpurun_out/n4probe/e_$np.txt; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/n4probe/l_$np.json'));print($np,d['ms_per_step'],d['roofline'].get('avg_ms'))"
done
