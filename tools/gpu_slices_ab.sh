# interleaved cold A/B of dl_shard_reduce_sgd between two library builds (build_ab/lib_{a,b}.so)
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
for T in t125 t1.3b; do for i in 1 2 3; do for v in a b; do
DILOCO_HIP_LIB=$R/build_ab/lib_$v.so timeout -k 10 200 python tools/slices_ab.py $T 7 2>/dev/null | sed "s/^/$v: /" || exit 1
done; done; done
