# DESIGN §5 hypothesis test: config #5 with eight gloo processes on one GPU, interleaved runs
# without any wait before gloo's collectives (nostage) and with only a device-side system-scope
# L2 write-back (fence). usage: gpurun --timeout 1200 -- bash tools/gpu_fence_probe.sh
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 1080 python -u tools/bf16_n8_repeat.py ${K:-10} nostage fence > gpurun_out/fence_probe.txt 2> gpurun_out/fence_probe.err
rc=$?
cat gpurun_out/fence_probe.txt
[ $rc -eq 0 ] || { echo "exit $rc"; tail -20 gpurun_out/fence_probe.err; }
