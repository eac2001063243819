#!/usr/bin/env python3
"""Host-synchronising HIP API calls inside a time window of a rocprofv3 --hip-trace CSV.

    python tools/api_sync_count.py <hip_api_trace.csv> <window_start_ns> <window_end_ns> [out.json]

Counts, inside [start, end] (CLOCK_MONOTONIC ns, as tools/gradsync_trace.py prints them) and in
the whole trace, every call whose name contains "Synchronize" (hipStreamSynchronize,
hipDeviceSynchronize, hipEventSynchronize, ...) plus hipMemcpy* calls by name."""
import csv
import json
import sys
from collections import Counter


def main():
    path, w0, w1 = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    inside, total = Counter(), Counter()
    first = last = None
    for r in csv.DictReader(open(path)):
        fn = r.get("Function") or r.get("Kind") or ""
        t = int(r["Start_Timestamp"])
        first = t if first is None else min(first, t)
        last = t if last is None else max(last, t)
        if "Synchronize" in fn or fn.startswith("hipMemcpy"):
            total[fn] += 1
            if w0 <= t <= w1:
                inside[fn] += 1
    out = {"window_ns": [w0, w1], "trace_span_ns": [first, last],
           "window_inside_trace": bool(first is not None and first <= w0 and w1 <= last),
           "inside_window": dict(inside), "whole_trace": dict(total)}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
