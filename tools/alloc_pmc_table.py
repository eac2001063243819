#!/usr/bin/env python3
"""Per allocation instance of tools/alloc_pmc.py: the dl_delta_pack_sgd dispatches' mean
duration (kernel trace) beside their mean counter values (counter collection).

    python tools/alloc_pmc_table.py DIR [DIR ...]   (rocprofv3 -d dirs, run_* csv inside)
"""
import csv
import os
import sys
from collections import defaultdict


def table(d):
    dur = {}
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        if "DeltaPackSgd" in r["Kernel_Name"]:
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    cnt = defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if "DeltaPackSgd" in r["Kernel_Name"]:
            cnt[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(cnt)
    names = sorted(next(iter(cnt.values())))
    print(d, "dispatches", len(ids))
    print("inst  ms      " + "  ".join(n.replace("_sum", "")[-26:] for n in names))
    per = 23
    for i in range(len(ids) // per):
        grp = ids[i * per + 4:(i + 1) * per]  # skip the first step's mode and the warm-ups
        ms = sum(dur.get(j, 0) for j in grp) / len(grp)
        vals = [sum(cnt[j][n] for j in grp) / len(grp) for n in names]
        print(f"{i:4d}  {ms:.4f}  " + "  ".join(f"{v:26.4g}" for v in vals))


if __name__ == "__main__":
    for d in sys.argv[1:]:
        table(d)
