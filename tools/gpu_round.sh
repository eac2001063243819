# GPU tests + smoke + bench line, then the rocprofv3 profile set (kernel trace of the bench
# headline, every kernel via tools/kernel_driver.py, FETCH/WRITE counter passes)
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_check.sh || exit 1
bash $R/tools/gpu_profile.sh ${1:-t125} || exit 1
