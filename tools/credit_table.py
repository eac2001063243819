#!/usr/bin/env python3
"""DRAM credit stalls per hot-path kernel from one rocprofv3 --pmc pass (VERDICT r05
item 3): TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum / TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum (cycles the
L2's write / read requests to HBM waited for a memory-controller credit, summed over the L2
channels), TCC_TAG_STALL_sum and GRBM_GUI_ACTIVE (GPU busy cycles), averaged over a kernel's
launches, and each stall sum per busy cycle. A kernel whose write-credit stalls outweigh its
read-credit stalls many times over is waiting on the write path to HBM.

    python tools/credit_table.py <run_counter_collection.csv> <tree> [out.json]
"""
import csv
import json
import re
import sys
from collections import defaultdict

COUNTERS = ("GRBM_GUI_ACTIVE", "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum",
            "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "TCC_TAG_STALL_sum")


def short(name):
    m = re.search(r"k_walk<dl::\(anonymous namespace\)::(\w+)<([^>]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.search(r"(k_\w+)(<[^(]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    path, tree = sys.argv[1], sys.argv[2]
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> counter -> value
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] in COUNTERS:
            per[short(r["Kernel_Name"])][r["Dispatch_Id"]][r["Counter_Name"]] = float(
                r["Counter_Value"])
    out = {"tree": tree, "source": path, "counters": COUNTERS, "kernels": {}}
    for k, disp in per.items():
        rows = [d for d in disp.values() if all(c in d for c in COUNTERS)]
        if not rows:
            continue
        mean = {c: sum(d[c] for d in rows) / len(rows) for c in COUNTERS}
        g = mean["GRBM_GUI_ACTIVE"]
        if g < 5e6:  # setup kernels (fills, copies, table resolves)
            continue
        out["kernels"][k] = {
            "launches": len(rows), "gui_active_cycles": round(g),
            "wr_credit_stall_per_cycle": round(mean["TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"] / g, 3),
            "rd_credit_stall_per_cycle": round(mean["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] / g, 3),
            "tag_stall_per_cycle": round(mean["TCC_TAG_STALL_sum"] / g, 3)}
    text = json.dumps(out, indent=1)
    print(text)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
