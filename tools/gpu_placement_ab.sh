# the placement A/B (tools/placement_ab.py): build order, a first-allocation ballast, one arena
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for b in none keep free none keep free; do
  PLACEMENT_AB_BALLAST=$b timeout -k 10 200 python3 tools/placement_ab.py 3 50 lazy,device >> gpurun_out/placement_ab2.json 2>> gpurun_out/placement_ab2.err || { tail -20 gpurun_out/placement_ab2.err; exit 1; }
  echo "ballast $b" >> gpurun_out/placement_ab2.json
done
for ord in device_one,device lazy_one,lazy device,device_one; do
  timeout -k 10 200 python3 tools/placement_ab.py 3 50 $ord >> gpurun_out/placement_ab2.json 2>> gpurun_out/placement_ab2.err || { tail -20 gpurun_out/placement_ab2.err; exit 1; }
done
grep -v Gloo gpurun_out/placement_ab2.json
