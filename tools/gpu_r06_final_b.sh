# Round-6 final-code record set, part B: the default bench line (N = 1), rocprofv3
# --kernel-trace --stats of the headline command, and the N = 8 rehearsal (eight gloo ranks on
# the one GPU) at the bench's default deadline.
# usage: gpurun --timeout 1200 -- bash tools/gpu_r06_final_b.sh
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/final
timeout -k 10 420 python bench.py --detail gpurun_out/final/bench_detail_n1.json > gpurun_out/final/bench_n1.json 2> gpurun_out/final/bench_n1.err \
  || { echo "bench failed"; tail -40 gpurun_out/final/bench_n1.err; exit 1; }
cat gpurun_out/final/bench_n1.json
bash tools/gpu_prof_headline.sh > gpurun_out/final/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/final/prof.log; exit 1; }
tail -2 gpurun_out/final/prof.log
TAG=r06 LIMIT=480 bash tools/gpu_rehearse_n8.sh > gpurun_out/final/n8.log 2>&1 || { echo "n8 rehearsal failed"; tail -30 gpurun_out/final/n8.log; exit 1; }
head -c 600 gpurun_out/bench_n8_gloo_r06.json
