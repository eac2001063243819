# dl_unpack_sgd_q8 at T1.3B: q8_spread.py and the bench leg's timing (q8_method.py), each with
# and without rocprofv3 kernel tracing, in one call on one box.
# usage: gpurun --timeout 900 -- bash tools/gpu_q8_method.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python3 tools/q8_method.py t1.3b 12 > gpurun_out/q8m_bench.json 2> gpurun_out/q8m.err || { tail -20 gpurun_out/q8m.err; exit 1; }
cat gpurun_out/q8m_bench.json
timeout -k 10 200 python3 tools/q8_spread.py t1.3b 12 > gpurun_out/q8m_spread.json 2>> gpurun_out/q8m.err || { tail -20 gpurun_out/q8m.err; exit 1; }
cat gpurun_out/q8m_spread.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_q8m -o run --output-format csv -- python3 $R/tools/q8_method.py t1.3b 12 > $R/gpurun_out/q8m_bench_prof.json 2>> $R/gpurun_out/q8m.err || { tail -20 $R/gpurun_out/q8m.err; exit 1; }
cat $R/gpurun_out/q8m_bench_prof.json
cd $R && timeout -k 10 200 python3 tools/q8_method.py t1.3b 12 > gpurun_out/q8m_bench2.json 2>> gpurun_out/q8m.err || { tail -20 gpurun_out/q8m.err; exit 1; }
cat gpurun_out/q8m_bench2.json
