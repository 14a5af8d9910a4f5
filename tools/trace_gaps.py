#!/usr/bin/env python3
"""Per-kernel durations and the gaps between consecutive dispatches from a rocprofv3 --kernel-trace CSV
(kernel_trace.csv): for each kernel name, count / median / mean duration, and the median idle gap before it
(previous dispatch's end -> this dispatch's start, same queue).  usage: trace_gaps.py <kernel_trace.csv> [skip]"""
import csv
import statistics as st
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[skip:]
    dur, gap = defaultdict(list), defaultdict(list)
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][:70]
        dur[name].append((e - s) / 1000.0)
        if prev_end is not None:
            gap[name].append((s - prev_end) / 1000.0)
        prev_end = e
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1000.0
    print(f"{len(rows)} dispatches over {span:.1f} us")
    for n in sorted(dur, key=lambda k: -sum(dur[k])):
        d, g = dur[n], gap.get(n, [0.0])
        print(f"{n:70s} n={len(d):6d} dur med {st.median(d):6.2f} mean {st.mean(d):6.2f} min {min(d):6.2f} "
              f"| gap-before med {st.median(g):6.2f} mean {st.mean(g):6.2f}  total {sum(d):9.1f}")


if __name__ == "__main__":
    main()
