# the write-through AUTO policy: store-policy bit-identity tests, the flags sweep (auto row vs
# the others) and the tiled two-kernel step on both trees, then one default bench line
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 170 --timeout-method thread -k "store_policies or slotted or pack_sgd or tiled or micro" > gpurun_out/pytest_wt.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_wt.log; exit 1; }
tail -1 gpurun_out/pytest_wt.log
timeout -k 10 400 python tools/cold_sweep.py --tree t125 --rounds 15 --what flags,tiles --out gpurun_out/autowt_t125.json 2>/dev/null | grep -E "auto|wt_stores|nt_loads\+stores  |^step" || exit 1
timeout -k 10 400 python tools/cold_sweep.py --tree t1.3b --rounds 5 --what flags --out gpurun_out/autowt_t13b.json 2>/dev/null | grep -E "auto|wt_stores|nt_loads\+stores  " || exit 1
timeout -k 10 450 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print('bench',d['value'],d['value_cold'],r['frac'],r.get('frac_vs_copy'),r.get('frac_vs_mix'))"
