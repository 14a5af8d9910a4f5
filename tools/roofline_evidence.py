"""Turn one tools/profile_round.sh run into the round's committed evidence under profiles/.

usage: python tools/roofline_evidence.py gpurun_out rNN

  profiles/<rNN>_bench_dnn4.json              the bench line of that run
  profiles/<rNN>_bench_dnn4_kernel_stats.csv  rocprofv3 --kernel-trace --stats summary (same command)
  profiles/<rNN>_rocprof_roofline.json        per-dispatch durations of the roofline kernel set (the
                                              2048x2048 fwd / bwd / update GEMMs) from the kernel
                                              trace, next to the bench's live hipEvent average
  profiles/<rNN>_pmc_gemm2048.json            HBM traffic per launch of the same kernel set from the
                                              FETCH_SIZE and WRITE_SIZE passes (tools/gemm_pmc.py
                                              layer), FETCH_SIZE doubled on gfx950 (MI355X_MICROARCH.md)
bench.py reads the newest profiles/r*_pmc_gemm2048.json for roofline.traffic.

The 2048x2048 launches are found in the trace by dispatch order inside each step (split at the
cache gather, or the update launch that carries it): forward = the three 64x128 BIAS_SIG launches after the K=440 layer; backward = the
diff-sigmoid launches except the first after softmax_xent (that one has K=4000); update = the
64-tile-row SGD launches with grid 65536 (the 4000-wide update has a larger grid).
"""
import csv
import json
import os
import re
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# (round 3: a trailing ", true" = the exact-prefetch instantiation, PX)
# (round 4: the form parameter SP -- 0 the LDS ring, 3..9 the direct forms -- and the pair kernel's forms of its
# update half and its backward half)
FWD = re.compile(r"gemm16_kernel<64, 128, 64, 2, 2, 2, \d+, true, false, 2(, (true|false))?>")    # bias + sigmoid
# (round 5: the backward from the transposed weight shadow is NN -- B n-contiguous -- in both)
BWD = re.compile(r"gemm16_kernel<64, 128, 64, 2, 2, 2, \d+, true, (true|false), 8(, (true|false))?>")  # diff-sigmoid + sums
PAIR = re.compile(r"gemm16_pair_kernel<128, 128, false, false, 9, (true|false), 64, 128, true, (true|false), 8, true(, \d+)*>")
UPD = re.compile(r"gemm16_kernel<128, 128, 64, 2, 2, 2, \d+, false, false, 9(, (true|false))?>")  # SGD + bias SGD


def classify_trace(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    cls = {"fwd": [], "bwd": [], "upd": [], "pair": []}
    after_softmax = False
    after_gather = False
    for r in rows:
        name = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        grid = int(r["Grid_Size_X"])
        if "softmax_xent" in name:
            after_softmax = True
            continue
        # the top layer's backward (K = 4000) with its own slab sums, round 3+: gemm16_bwd_slabs_kernel -- then
        # the next diff-sigmoid launch is the 2048^2 backward (the plain BWD below), not the K = 4000 one
        if "gemm16_bwd_slabs_kernel" in name:
            after_softmax = False
            continue
        # the bunch gather: its own launch, or (round 3, tnet_affine_update_bias_gather) riding on the
        # previous step's last update launch (the 440x2048 update, not a roofline GEMM)
        # (round 4: the last two updates + the gather, gemm16_upd_mixed_gather_kernel -- not a roofline launch)
        if "gather_rows" in name or "upd_gather" in name or "upd_mixed_gather" in name:
            after_gather = True
            continue
        if FWD.search(name):
            if after_gather:           # K = 440 (the first layer, same tile config)
                after_gather = False
            else:
                cls["fwd"].append(dur)
        elif BWD.search(name):
            if after_softmax:          # K = 4000 (error into the last hidden layer)
                after_softmax = False
            else:
                cls["bwd"].append(dur)
        elif UPD.search(name) and grid == 65536:
            cls["upd"].append(dur)
        elif PAIR.search(name) and grid == 2 * 65536:
            # round 3: a 2048x2048 update + the 2048x2048 backward of the layer below in one launch
            # (tnet_affine_update_bwd_pair): two GEMMs, each counted at half the launch
            cls["pair"] += [dur / 2, dur / 2]
    return cls


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
    with open(os.path.join(prof, f"{tag}_bench_dnn4.json"), "w") as f:
        json.dump(bench, f, indent=1)
    shutil.copyfile(os.path.join(src, "prof_stats", "bench_kernel_stats.csv"),
                    os.path.join(prof, f"{tag}_bench_dnn4_kernel_stats.csv"))
    cls = classify_trace(os.path.join(src, "prof_stats", "bench_kernel_trace.csv"))
    allv = cls["fwd"] + cls["bwd"] + cls["upd"] + cls["pair"]
    prof_bench = json.loads(open(os.path.join(src, "bench_prof.json")).read().strip().splitlines()[-1])
    tr = {"source": "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline",
          "per_class_avg_us": {k: round(sum(v) / len(v), 2) for k, v in cls.items() if v},
          "per_class_launches": {k: len(v) for k, v in cls.items()},
          "roofline_set_avg_us_rocprof": round(sum(allv) / len(allv), 2),
          "roofline_set_avg_us_hipevent_same_run": prof_bench["roofline"]["avg_launch_us"],
          "roofline_set_avg_us_hipevent_bench_run": bench["roofline"]["avg_launch_us"],
          "note": "warmup launches included in the rocprof average (the trace covers the whole process)"}
    with open(os.path.join(prof, f"{tag}_rocprof_roofline.json"), "w") as f:
        json.dump(tr, f, indent=1)
    fetch = pmc_summary.summarise(os.path.join(src, "pmc_fetch"))
    write = pmc_summary.summarise(os.path.join(src, "pmc_write"))
    kern = {}
    for d in (fetch, write):
        for k, r in d.items():
            if "gemm" in k:
                kern.setdefault(k, {}).update({kk: v for kk, v in r.items() if kk in ("kernel", "grid", "dispatches",
                                                                                       "fetch_MB_x2", "write_MB")})
    per = [r["fetch_MB_x2"] + r["write_MB"] for r in kern.values()]
    algo = {"fwd": (1024 * 2048 + 2048 * 2048 + 1024 * 2048) * 4 / 1e6,     # X, W read; Y written
            "bwd": (1024 * 2048 * 3 + 2048 * 2048) * 4 / 1e6,               # E, W, Ybelow read; Eo written
            "upd": (1024 * 2048 * 2 + 2048 * 2048 * 2) * 4 / 1e6}           # X, E read; W read + written
    pmc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- python3 "
                     "tools/gemm_pmc.py layer 20; FETCH_SIZE x2 (gfx950), KiB -> MB",
           "kernels": kern, "traffic_MB_per_launch": round(sum(per) / len(per), 3),
           "algorithmic_MB_per_launch": {k: round(v, 3) for k, v in algo.items()},
           "algorithmic_MB_per_launch_avg": round(sum(algo.values()) / 3, 3)}
    # MFMA utilisation pass (GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F32) and
    # the in-kernel clock stamps (tools/gemm_clock.py, separate stamped build)
    if os.path.isdir(os.path.join(src, "pmc_mfma")):  # optional passes (a round may skip them)
        mf = pmc_summary.summarise(os.path.join(src, "pmc_mfma"))
        pmc["mfma_pass"] = {k: r for k, r in mf.items() if "gemm" in k}
        pmc["mfma_pass_note"] = ("mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs); "
                                 "GRBM_GUI_ACTIVE/8/duration reads above the real clock on sub-0.3-ms dispatches "
                                 "(MI355X_MICROARCH.md 'DVFS give-back'), so the in-kernel stamps below are the "
                                 "clock and cycle reference")
    clk = [l for l in open(os.path.join(src, "clock.log")) if l.startswith("CLOCK ")] \
        if os.path.exists(os.path.join(src, "clock.log")) else []
    if clk:
        pmc["clock_stamps"] = json.loads(clk[-1][6:])
    with open(os.path.join(prof, f"{tag}_pmc_gemm2048.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    print(json.dumps(tr, indent=1))
    print(json.dumps(pmc, indent=1))


if __name__ == "__main__":
    main()
