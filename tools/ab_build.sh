# Build two variants of libdiloco_hip.so for an interleaved A/B on one GPU box
# (tools/gpu_ab.sh runs the kernel tests on variant b, then tile_ab / sweep on a, b, a, b ...).
#   bash tools/ab_build.sh "<hipcc flags of a>" "<hipcc flags of b>"   e.g. "" "-DMY_VARIANT"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/build_ab"
cd "$R/diloco-swarm_amd/csrc"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fvisibility=hidden -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -Wall -Wno-unused-function"
SRC="dl_kernels.hip dl_q8.hip dl_xgmi.hip dl_comm.hip dl_abi.hip"
/opt/rocm/bin/hipcc $F $1 $SRC -ldl -o "$R/build_ab/lib_a.so"
/opt/rocm/bin/hipcc $F $2 $SRC -ldl -o "$R/build_ab/lib_b.so"
