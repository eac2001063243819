# re-check the write-through vs non-temporal store choice with the
# flushed cold timing (tools/cold_sweep.py --flushed: each launch charged with the HBM
# write-back of the lines it leaves dirty). Product library: "auto" is write-through for
# dl_unpack_sgd_q8 below 2^28 elements, "nt_loads+stores" the NT policy; the fp32 kernels'
# AUTO (plain / NT stores) against the other product policy.
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out/flushed
for T in t125 t1.3b; do
  timeout -k 10 400 python tools/cold_sweep.py --tree $T --rounds 7 --what q8,flags --flushed --out gpurun_out/flushed/sweep_$T.json > gpurun_out/flushed/sweep_$T.txt 2>&1 || { echo sweep $T failed; tail gpurun_out/flushed/sweep_$T.txt; exit 1; }
  echo "== $T"; grep -E "auto|nt_loads\+stores  |nt_loads  " gpurun_out/flushed/sweep_$T.txt
done
