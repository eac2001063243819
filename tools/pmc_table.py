#!/usr/bin/env python3
"""Per-kernel averages of every counter in one or more rocprofv3 --pmc counter_collection CSVs
(values summed over each dispatch's dimensions, then averaged over the kernel's dispatches),
plus derived figures where their counters are present:
    ea_rd_latency_cycles  = TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ   (Little's law, per request)
    ea_wr_latency_cycles  = TCC_EA0_WRREQ_LEVEL / TCC_EA0_WRREQ
    l2_hit                = TCC_HIT / (TCC_HIT + TCC_MISS)
    *_frac                = a stall / busy cycle count over TCC_BUSY, GRBM_GUI_ACTIVE, TA/TD
                            busy or SQ_WAVE_CYCLES (see the keys)

    python tools/pmc_table.py out.json a.csv [b.csv ...]
"""
import csv
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import short  # noqa: E402


def load(paths):
    per = defaultdict(float)  # (kernel, dispatch, counter) -> value
    for path in paths:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            k = short(name) or ("copy" if "k_copy<true" in name else
                                "scrub" if "k_copy<false" in name else None)
            if k is None:
                continue
            per[(k, path + r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(list))
    for (k, _d, c), v in per.items():
        agg[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def derive(c):
    d = {}

    def ratio(name, num, den):
        if num in c and den in c and c[den]:
            d[name] = round(c[num] / c[den], 4)

    ratio("ea_rd_latency_cycles", "TCC_EA0_RDREQ_LEVEL", "TCC_EA0_RDREQ")
    ratio("ea_wr_latency_cycles", "TCC_EA0_WRREQ_LEVEL", "TCC_EA0_WRREQ")
    if "TCC_HIT" in c and "TCC_MISS" in c and (c["TCC_HIT"] + c["TCC_MISS"]):
        d["l2_hit"] = round(c["TCC_HIT"] / (c["TCC_HIT"] + c["TCC_MISS"]), 4)
    for s in ("TCC_EA0_WRREQ_STALL", "TCC_TOO_MANY_EA_WRREQS_STALL",
              "TCC_EA0_WRREQ_DRAM_CREDIT_STALL", "TCC_EA0_RDREQ_DRAM_CREDIT_STALL",
              "TCC_TAG_STALL"):
        ratio(s.lower() + "_per_busy", s, "TCC_BUSY")
    ratio("ta_busy_per_gui", "TA_TA_BUSY", "GRBM_GUI_ACTIVE")
    ratio("ta_addr_stalled_by_tc_per_ta_busy", "TA_ADDR_STALLED_BY_TC_CYCLES", "TA_TA_BUSY")
    ratio("td_tc_stall_per_td_busy", "TD_TC_STALL", "TD_TD_BUSY")
    ratio("sq_wait_any_per_wave_cycle", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES")
    return d


def main():
    out, paths = sys.argv[1], sys.argv[2:]
    t = load(paths)
    res = {k: {"counters": {c: round(v, 1) for c, v in sorted(cs.items())}, "derived": derive(cs)}
           for k, cs in sorted(t.items())}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, r in res.items():
        print(k, json.dumps(r["derived"]))


if __name__ == "__main__":
    main()
