#!/usr/bin/env python3
"""Summarise bench.py's compact lines from a scaling run (one JSON line per N: the driver's
SCALE_rNN.json, or several bench outputs) against the N > 1 model of DESIGN.md §4: the headline
(the reference's calls on the sharded exchange), its exchange roofline, the exchange efficiency
per tree (the step's bus rate over RCCL's own all_reduce of the same bytes), every leg's GB/s and
HBM bytes per parameter, and the parity self-checks, per N.

    python tools/scale_report.py SCALE_r04.json [more files ...]
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
    base = None
    print(" | ".join(("N", "headline GB/s", "aggregate", "ms/step", "eff vs N=1", "xchg frac",
                      "eff t125", "eff t1.3b", "model@76.8")))
    for d in rows:
        n = d.get("n_gpus") or 1
        if n == 1:
            base = d.get("value")
        ee = d.get("exchange_efficiency") or {}
        agg = d.get("value_aggregate")
        eff = agg / (n * base) if agg and base else None
        row = (n, d.get("value"), agg, d.get("ms_per_step"), eff,
               val(d, "roofline", "frac") if n > 1 else None,
               val(ee, "t125", "frac_of_rccl_allreduce"),
               val(ee, "t1.3b", "frac_of_rccl_allreduce"), model_gbs(n))
        print(" | ".join("-" if x is None else (f"{x:.3f}" if isinstance(x, float) else str(x))
                         for x in row))
        for k, v in sorted((d.get("legs") or {}).items()):
            print(f"    {k}: {v.get('GBs')} GB/s, {v.get('ms')} ms, frac {v.get('frac')}, "
                  f"{v.get('Bpp')} B/param")
        bad = [k for k, v in (d.get("parity") or {}).items() if not v.get("ok")]
        print(f"    parity: {'all ok' if not bad else 'FAILED ' + ', '.join(bad)}")
        if d.get("skipped_legs") or d.get("incomplete"):
            print(f"    skipped {d.get('skipped_legs')} incomplete {d.get('incomplete')}")


if __name__ == "__main__":
    main()
