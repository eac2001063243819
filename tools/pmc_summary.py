#!/usr/bin/env python3
"""Per-launch HBM bytes of the outer-step kernels from rocprofv3 --pmc passes.

    python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
        <tree> <out.json>

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports exactly half the bytes
of a wide coalesced streaming read -> x2. WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.
Counters are summed over the dimensions rocprofv3 reports per dispatch, then averaged over the
dispatches of each kernel.
"""
import csv
import re
import json
import sys
from collections import defaultdict


def short(name):
    # most specific first: k_flat<UnpackSgd...> is dl_shard_sgd, UnpackSgdQ8 is not UnpackSgd
    names = {"k_xgmi_reduce_sgd": "xgmi_reduce_sgd", "k_flat": "shard_sgd", "DeltaQ8": "delta_q8", "UnpackSgdQ8": "unpack_sgd_q8",
             "k_q8_reduce": "q8_reduce", "DeltaPackSgd": "delta_pack_sgd",
             "DeltaPackPair": "delta_pack_pairs", "GatherPair": "gather_pairs",
             "DeltaPack": "delta_pack", "UnpackSgd": "unpack_sgd",
             "UnpackAvg": "unpack_avg", "DeltaSgd": "delta_sgd", "Gather": "gather",
             "Scatter": "scatter", "k_fill_synth": "fill_synth",
             "k_serialize_f32x4": "serialize_f32", "k_serialize<unsigned short>": "serialize_bf16",
             "k_slices_sgd": "shard_reduce_sgd"}
    if "k_xgmi_reduce_sgd" in name and ", true>" in name:
        return "xgmi_delta_sgd"  # the pack-free variant (exchange="xgmi_inner")
    for k, v in names.items():
        if k in name:
            # the SGD bodies' MODE (1 = first step) is the last argument of the body's own
            # template list (k_walk's trailing arguments are the load / store policy)
            body = "UnpackSgd" if k == "k_flat" else k
            m = re.search(re.escape(body) + r"<([^<>]*)>", name)
            first = (k in ("UnpackSgd", "k_flat", "DeltaSgd", "DeltaPackSgd", "UnpackSgdQ8",
                           "k_slices_sgd")
                     and m is not None and m.group(1).split(",")[-1].strip() == "1")
            if k == "k_slices_sgd" and m is not None:  # the slice count is its first argument
                nsl = m.group(1).split(",")[0].strip()
                v += "" if nsl == "1" else f"_n{nsl}"
            return v + ("_first" if first else "")
    return None


def load(path, counter):
    per = defaultdict(float)  # (kernel, dispatch) -> value
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        k = short(r["Kernel_Name"])
        if k is None:
            continue
        per[(k, r["Dispatch_Id"])] += float(r["Counter_Value"])
    agg = defaultdict(list)
    for (k, _d), v in per.items():
        agg[k].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    fpath, wpath, tree, out = sys.argv[1:5]
    f = load(fpath, "FETCH_SIZE")
    w = load(wpath, "WRITE_SIZE")
    res = {"tree": tree, "unit": "bytes per launch", "correction": "FETCH_SIZE x2 (gfx950)",
           "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fb = f.get(k, 0.0) * 1024 * 2
        wb = w.get(k, 0.0) * 1024
        res["kernels"][k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
