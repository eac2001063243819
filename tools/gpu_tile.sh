R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "tiled or ragged or micro" > gpurun_out/pytest_tile.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_tile.log; exit 1; }
tail -2 gpurun_out/pytest_tile.log
timeout -k 10 300 python tools/tile_ab.py --tree t125 --rounds 9 --out gpurun_out/tile_ab_t125.json > gpurun_out/tile_t125.txt 2>&1 || { echo tile failed; tail gpurun_out/tile_t125.txt; exit 1; }
cat gpurun_out/tile_t125.txt
timeout -k 10 300 python tools/tile_ab.py --tree t1.3b --rounds 5 --steps 4 --flags auto,plain --out gpurun_out/tile_ab_t13b.json > gpurun_out/tile_t13b.txt 2>&1 || { echo tile13 failed; tail gpurun_out/tile_t13b.txt; exit 1; }
cat gpurun_out/tile_t13b.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --deadline 12 > gpurun_out/bench_wd.json 2> gpurun_out/bench_wd.err; echo "wd rc=$?"; cat gpurun_out/bench_wd.json; tail -5 gpurun_out/bench_wd.err
