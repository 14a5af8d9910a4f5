#!/usr/bin/env python3
"""Collect bench.py A/B runs (one JSON line per file) into one evidence file: per arm the values, steps, roofline
fractions and the per-kernel event-timed averages of every run.

usage: python tools/collect_ab.py OUT.json "what was compared" ARM=glob [ARM=glob ...]"""
import glob
import json
import statistics
import sys


def last_json(path):
    rows = [l for l in open(path) if l.lstrip().startswith("{")]
    return json.loads(rows[-1]) if rows else None


def main():
    out, what, arms = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = {"what": what, "arms": {}}
    for spec in arms:
        name, pat = spec.split("=", 1)
        runs = [r for r in (last_json(p) for p in sorted(glob.glob(pat))) if r]
        if not runs:
            raise SystemExit(f"{name}: no runs match {pat}")
        kern = {}
        for r in runs:
            for k, v in (r.get("kernels") or {}).items():
                kern.setdefault(k, []).append(v["avg_us"])
        res["arms"][name] = {
            "files": sorted(glob.glob(pat)),
            "workload": runs[0]["config"].get("workload"),
            "values": [r["value"] for r in runs], "median_value": statistics.median(r["value"] for r in runs),
            "ms_per_step": [r["ms_per_step"] for r in runs],
            "roofline_frac": [r.get("roofline", {}).get("frac") for r in runs],
            "kernel_avg_us_median": {k: round(statistics.median(v), 2) for k, v in sorted(kern.items())},
        }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v["median_value"] for k, v in res["arms"].items()}))


if __name__ == "__main__":
    main()
