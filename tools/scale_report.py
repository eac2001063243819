#!/usr/bin/env python3
"""Summarise bench.py lines from a scaling run (one JSON line per N: the driver's
SCALE_rNN.json, or several bench outputs) against the N > 1 model of DESIGN.md §4: headline
(RCCL sharded step), the replicated all-reduce variant, 64 MiB buckets, the ordered a2a step,
the direct peer-access exchange, RCCL's own all_reduce busBW, the per-step grad sync (all_reduce
and a2a), the RCCL setting variants and the link probe, per N.

    python tools/scale_report.py SCALE_r01.json [more files ...]
"""
import json
import sys

P_T125 = 124475904


def lines(paths):
    for p in paths:
        with open(p) as f:
            text = f.read()
        try:  # one JSON document: a list of lines, {N: line}, or wrapper objects
            doc = json.loads(text)
        except ValueError:
            doc = None
        if doc is not None:
            items = doc if isinstance(doc, list) else list(doc.values()) if isinstance(
                doc, dict) and "metric" not in doc else [doc]
            for it in items:
                if isinstance(it, dict) and "metric" in it:
                    yield it
                elif isinstance(it, dict):
                    yield from (v for v in it.values() if isinstance(v, dict) and "metric" in v)
            continue
        for ln in text.splitlines():
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                yield json.loads(ln)


def val(d, *keys):
    for k in keys:
        if not isinstance(d, dict):
            return None
        d = d.get(k)
    return d


def model_gbs(n, link=76.8):
    """value = 4P/t with t = 2(n-1)/n·4P / ((n-1)·L): every link at L GB/s per
    direction."""
    if n <= 1:
        return None
    t = 2 * (n - 1) / n * 4 * P_T125 / ((n - 1) * link * 1e9)
    return 4 * P_T125 / t / 1e9


def main():
    rows = sorted(lines(sys.argv[1:]), key=lambda d: d.get("n_gpus", 0))
    hdr = ("N", "headline", "ms/step", "allreduce var", "64MiB", "a2a", "xgmi", "xgmi parity",
           "rccl AR busBW", "frac of AR", "grad sync", "grad sync a2a", "link 1-peer",
           "model@76.8")
    print(" | ".join(hdr))
    for d in rows:
        n = d.get("n_gpus") or 1
        e = d.get("extra") or {}
        p = d.get("parity") or {}
        row = (n, d.get("value"), d.get("ms_per_step"),
               val(e, "t125_allreduce_variant", "value"), val(e, "t125_bucket64MiB", "value"),
               val(e, "t125_a2a", "value"),
               val(e, "t125_xgmi_exchange", "value"), val(p, "xgmi", "ok"),
               val(e, "rccl_allreduce_ref", "all_reduce", "busbw_GBs"),
               val(d, "exchange_efficiency", "frac_of_rccl_allreduce"),
               val(e, "t125_dp_grad_sync", "value"), val(e, "t125_dp_grad_sync_a2a", "value"),
               val(e, "xgmi_link_probe", "one_peer_read_GBs"), model_gbs(n))
        print(" | ".join("-" if x is None else (f"{x:.1f}" if isinstance(x, float) else str(x))
                         for x in row))
        for k in sorted(e):
            if k.startswith("rccl_env_"):
                print(f"    {k}: step {val(e, k, 'sharded_step', 'value')} GB/s, AR busBW "
                      f"{val(e, k, 'rccl_allreduce_ref', 'all_reduce', 'busbw_GBs')}")
        for k in sorted(d):
            if k.startswith("exchange_efficiency_"):
                print(f"    {k}: {d[k]}")
        for k in ("t1.3b", "t1.3b_bf16_wire", "t1.3b_bf16_a2a", "t1.3b_int8_wire"):
            if val(e, k, "value") is not None:
                print(f"    {k}: {val(e, k, 'value')} GB/s, {val(e, k, 'ms_per_step')} ms/step")
        for k in ("a2a", "a2a_bf16", "sharded", "bf16"):
            if isinstance(p.get(k), dict):
                print(f"    parity {k}: ok={p[k].get('ok')} identical={p[k].get('replicas_identical')}")
        if d.get("skipped_legs") or d.get("incomplete"):
            print(f"    skipped {d.get('skipped_legs')} incomplete {d.get('incomplete')}")


if __name__ == "__main__":
    main()
