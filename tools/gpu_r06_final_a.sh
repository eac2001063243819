# Round-6 final-code record set, part A (one GPU call): the T125 PMC passes of the hot-path
# kernels (FETCH_SIZE, WRITE_SIZE in separate runs -> the traffic the bench line carries),
# every -m gpu test once (not stopping at a failure: the record shows all), smoke().
# usage: gpurun --timeout 1200 -- bash tools/gpu_r06_final_a.sh
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/final
if [ -z "$SKIP_PMC" ]; then  # SKIP_PMC=1: the tests and smoke() only
  bash tools/gpu_pmc.sh t125 > gpurun_out/final/pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/final/pmc.log; exit 1; }
  cp gpurun_out/pmc_t125.json gpurun_out/final/r06_pmc_t125.json
fi
cd $R
DILOCO_TEST_RECORD=$R/gpurun_out/final/eight_peer_gpu_state.jsonl \
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rw --timeout 400 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/final/pytest_gpu.txt 2>&1
rc=$?
tail -3 gpurun_out/final/pytest_gpu.txt
[ $rc -le 1 ] || { echo "pytest ended with $rc: stopping"; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.txt 2>&1 \
  || { echo "smoke failed"; tail -30 gpurun_out/final/smoke.txt; exit 1; }
tail -2 gpurun_out/final/smoke.txt
exit $rc
