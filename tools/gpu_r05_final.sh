# Round-5 final-code record set (one GPU call): every -m gpu test (not stopping at the first
# failure: the record shows all of them), smoke(), and the default bench line.
# usage: gpurun --timeout 1200 -- bash tools/gpu_r05_final.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 780 python -u -m pytest tests -m gpu -q -rw --timeout 400 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_final.log
[ $rc -le 1 ] || { echo "pytest ended with $rc: stopping"; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 \
  || { echo "smoke failed"; tail -30 gpurun_out/smoke_final.log; exit 1; }
tail -2 gpurun_out/smoke_final.log
timeout -k 10 420 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err \
  || { echo "bench failed"; tail -40 gpurun_out/bench_final.err; exit 1; }
cat gpurun_out/bench_final.json
