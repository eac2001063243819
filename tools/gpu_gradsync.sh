# per-step DP grad sync over a one-rank RCCL group with reallocated grads: rate, then the same
# under rocprofv3 --hip-trace and the host-synchronising API calls inside the steady state
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 120 python tools/gradsync_trace.py t125 20 > gpurun_out/gradsync.json 2> gpurun_out/gradsync.err || { echo gradsync failed; tail gpurun_out/gradsync.err; exit 1; }
cat gpurun_out/gradsync.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --hip-trace --output-format csv -d $R/gpurun_out/gs_trace -o run -- python3 $R/tools/gradsync_trace.py t125 20 > $R/gpurun_out/gradsync_traced.json 2> $R/gpurun_out/gradsync_traced.err || { echo traced gradsync failed; tail $R/gpurun_out/gradsync_traced.err; exit 1; }
W=$(python3 -c "import json;d=json.loads(open('$R/gpurun_out/gradsync_traced.json').read().strip().splitlines()[-1]);print(*d['window_monotonic_ns'])")
T=$(find $R/gpurun_out/gs_trace -name "*hip_api_trace.csv" | head -1)
python3 $R/tools/api_sync_count.py $T $W $R/gpurun_out/gradsync_api_syncs.json
rm -f $T
