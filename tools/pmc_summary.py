"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (name + grid size).

usage: python tools/pmc_summary.py gpurun_out/pmc   -> table on stdout, JSON with --json

Units / corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section):
  FETCH_SIZE, WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE counts half the bytes of wide
  16-B/lane streaming reads (global_load_dwordx4 and LDS-DMA alike), so it is doubled here.
  GRBM_GUI_ACTIVE is summed over the 8 XCDs: effective clock = GRBM_GUI_ACTIVE / 8 / duration.
  SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs) = fraction of SIMD-cycles with an MFMA busy.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*$", "", name)
    n = n.replace("void ", "")
    return n[:90]


def load(d):
    per = defaultdict(lambda: defaultdict(list))  # (kernel, grid) -> counter -> [values]
    dur = defaultdict(dict)                         # (kernel, grid) -> {dispatch: ns}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            key = (short(row["Kernel_Name"]), int(row["Grid_Size"]))
            per[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
            dur[key][(f, row["Dispatch_Id"])] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    return per, dur


def summarise(d):
    per, dur = load(d)
    out = {}
    for key, cs in per.items():
        ds = list(dur[key].values())
        avg_ns = sum(ds) / len(ds)
        r = {"kernel": key[0], "grid": key[1], "dispatches": len(ds), "avg_us_profiled": avg_ns / 1e3}
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in mean:
            r["fetch_MB_x2"] = mean["FETCH_SIZE"] * 1024 * 2 / 1e6
        if "WRITE_SIZE" in mean:
            r["write_MB"] = mean["WRITE_SIZE"] * 1024 / 1e6
        if "GRBM_GUI_ACTIVE" in mean:
            # duration of the SQ pass dispatches only (the counter pass that holds GRBM)
            r["eff_clock_GHz"] = mean["GRBM_GUI_ACTIVE"] / 8 / avg_ns
            if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
                # rocprofv3's MfmaUtil: busy cycles summed over the SIMDs / (GRBM cycles x SIMD count)
                r["mfma_busy_frac"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (mean["GRBM_GUI_ACTIVE"] / 8 * 1024)
            if "SQ_INSTS_VALU_MFMA_MOPS_F32" in mean:
                r["mfma_flops_f32"] = mean["SQ_INSTS_VALU_MFMA_MOPS_F32"] * 512
        for c in ("SQ_BUSY_CU_CYCLES", "SQ_WAVES"):
            if c in mean:
                r[c] = mean[c]
        out[f"{key[0]}|{key[1]}"] = r
    return out


if __name__ == "__main__":
    d = sys.argv[1]
    res = summarise(d)
    if "--json" in sys.argv:
        print(json.dumps(res, indent=1))
    else:
        rows = sorted(res.values(), key=lambda r: -r["avg_us_profiled"] * r["dispatches"])
        for r in rows:
            print(f'{r["kernel"][:60]:60s} grid={r["grid"]:>9d} n={r["dispatches"]:4d} '
                  f'{r["avg_us_profiled"]:8.1f}us ' + " ".join(f"{k}={v:.3f}" for k, v in r.items()
                                                            if k not in ("kernel", "grid", "dispatches", "avg_us_profiled")))
