# Producer -> consumer pairs, flushed cold (each launch charged with its dirty-line write-back):
# plain vs non-temporal stores where the next kernel re-reads the output (tools/cold_sweep.py
# pipe), T125 and T1.3B; then the bf16 drop-in GPU test.
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out/pipe
for T in t125 t1.3b; do
  timeout -k 10 300 python tools/cold_sweep.py --tree $T --rounds 9 --what pipe --flushed --out gpurun_out/pipe/pipe_$T.json > gpurun_out/pipe/pipe_$T.txt 2>&1 || { echo pipe $T failed; tail gpurun_out/pipe/pipe_$T.txt; exit 1; }
  echo "== $T"; grep -E "med" gpurun_out/pipe/pipe_$T.txt
done
