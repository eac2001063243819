#!/usr/bin/env python3
"""Per-kernel table from a rocprofv3 --stats kernel summary and the matching PMC summary:
average duration, algorithmic bytes per launch (given per parameter below), achieved GB/s,
fraction of the 8 TB/s HBM3E peak and measured HBM bytes (FETCH x2 + WRITE) per launch.

    python tools/kernel_table.py <run_kernel_stats.csv> <pmc_<tree>.json> <tree> [out.json]
"""
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))
sys.path.insert(0, HERE)

from pmc_summary import short  # noqa: E402

PEAK = 8000.0
Q8_SLOT, CHUNK = 4160, 4096
ACT = 32 * 1024 * 768  # the Serializer's (32, 1024, 768) activation


def algorithmic(kernel, P, n_chunks):
    slot = n_chunks * Q8_SLOT
    table = {"delta_pack": 12 * P, "unpack_sgd": 24 * P, "unpack_sgd_first": 20 * P,
             "delta_sgd": 24 * P, "delta_sgd_first": 20 * P, "delta_pack_sgd": 28 * P,
             "delta_pack_sgd_first": 24 * P, "gather": 8 * P, "scatter": 8 * P,
             "unpack_avg": 8 * P, "shard_sgd": 20 * P, "shard_sgd_first": 16 * P,
             "delta_q8": 8 * P + slot, "q8_reduce": 2 * slot,
             "unpack_sgd_q8": slot + 20 * P, "unpack_sgd_q8_first": slot + 16 * P,
             "xgmi_reduce_sgd": 20 * P, "xgmi_delta_sgd": 20 * P,
             "serialize_f32": 8 * ACT, "serialize_bf16": 6 * ACT,
             # n = 1 (the whole tree, 20 B); n = 8: 8 fp32 slices of an eighth + θ, buf
             "shard_reduce_sgd": 20 * P, "shard_reduce_sgd_first": 16 * P,
             "shard_reduce_sgd_n8": (P // 8 // 64 * 64) * (8 * 4 + 16),
             "shard_reduce_sgd_n8_first": (P // 8 // 64 * 64) * (8 * 4 + 12)}
    return table.get(kernel)


def main():
    stats, pmc_path, tree = sys.argv[1:4]
    from diloco_amd.trees import get_tree

    spec = get_tree(tree)
    P = spec.total()
    n_chunks = sum(-(-n // CHUNK) for n in spec.numels())
    pmc = json.load(open(pmc_path))["kernels"]
    rows = {}
    for r in csv.DictReader(open(stats)):
        k = short(r["Name"])
        if k is None or k == "fill_synth":
            continue
        ms = float(r["AverageNs"]) / 1e6
        b = algorithmic(k, P, n_chunks)
        if b is None:
            continue
        e = rows.setdefault(k, {"calls": 0, "ns": 0.0})
        e["calls"] += int(r["Calls"])
        e["ns"] += float(r["TotalDurationNs"])
    out = {}
    for k, e in sorted(rows.items()):
        ms = e["ns"] / e["calls"] / 1e6
        b = algorithmic(k, P, n_chunks)
        gbs = b / (ms * 1e-3) / 1e9
        hbm = pmc.get(k, {}).get("hbm_bytes")
        out[k] = {"calls": e["calls"], "avg_us": round(ms * 1e3, 1), "bytes": b,
                  "GBs": round(gbs, 1), "frac": round(gbs / PEAK, 3),
                  "pmc_over_alg": round(hbm / b, 4) if hbm else None}
        print(f"{k:22s} calls {e['calls']:3d} avg {ms*1e3:9.1f} us  {gbs:7.1f} GB/s  "
              f"{gbs/PEAK:.3f}  pmc/alg {out[k]['pmc_over_alg']}")
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            json.dump({"tree": tree, "params": P, "peak_GBs": PEAK, "kernels": out}, f, indent=1)


if __name__ == "__main__":
    main()
