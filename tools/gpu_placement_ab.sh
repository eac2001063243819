# the placement A/B (tools/placement_ab.py) in both build orders, each its own process
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for ord in lazy,device device,lazy lazy,device device,lazy; do
  timeout -k 10 200 python3 tools/placement_ab.py 3 50 $ord >> gpurun_out/placement_ab.json 2>> gpurun_out/placement_ab.err || { tail -20 gpurun_out/placement_ab.err; exit 1; }
done
grep -v Gloo gpurun_out/placement_ab.json
