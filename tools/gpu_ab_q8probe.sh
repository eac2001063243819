# int8 encoder probe: the quantiser's IEEE division (q0) vs a reciprocal multiply (q1) vs no
# quantiser arithmetic (q2), cold, interleaved across processes (tools/cold_sweep.py q8)
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
for i in 1 2; do for v in q0 q1 q2; do for t in t125 t1.3b; do
DILOCO_HIP_LIB=$R/build_ab/lib_$v.so timeout -k 10 200 python tools/cold_sweep.py --tree $t --rounds 7 --what q8 --out gpurun_out/probe_${v}_${t}_$i.json 2>/dev/null | sed "s/^/$v $t: /" || exit 1
done; done; done
