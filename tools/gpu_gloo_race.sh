# usage: gpurun --timeout 600 -- bash tools/gpu_gloo_race.sh   (RACE_* env: sizes, variants)
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 tools/gloo_race.py > gpurun_out/gloo_race.txt 2> gpurun_out/gloo_race.err || { tail -30 gpurun_out/gloo_race.err; exit 1; }
grep bad_elements gpurun_out/gloo_race.txt
