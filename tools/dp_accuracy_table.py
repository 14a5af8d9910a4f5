#!/usr/bin/env python3
"""Build profiles/r05_dp_accuracy_ex01.json: frame accuracy of every data-parallel mode on
examples/01's MLP3 (5 seeds each; round 4's N = 1 / strong / weak points from profiles/r04_dp_accuracy_ex01.json,
round 5's middle points -- 256 and 512 rows a rank at N = 8 -- from tools/gpurun_batches/r5d.sh's logs) beside the
one-rank data-parallel step time at that bunch (bench.py --config mlp3 --force-dp --bunch B, the N > 1 path's own
cost on one GPU) and the N = 8 throughput that step time allows.

The N = 8 projection is a BOUND, not a measurement (one GPU per call here): 8 B / (t_dp(B) + t_ar), t_ar = the
3.24 MB all-reduce of MLP3's gradients over 8 GPUs, which this box cannot time; the table gives the bound at
t_ar = 0 and at an assumed t_ar (default 40 us: a ring all-reduce moves 2 (N - 1) / N x 3.24 MB = 5.7 MB a GPU,
~20 us at 300 GB/s of per-GPU xGMI bandwidth, plus ~20 us of RCCL launch / ring latency -- stated, not measured).

usage: python tools/dp_accuracy_table.py <r5d dir> <bench dir> [t_ar_us] > profiles/r05_dp_accuracy_ex01.json
"""
import glob
import json
import os
import re
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def last_json(path):
    rows = [l for l in open(path) if l.lstrip().startswith("{")]
    return json.loads(rows[-1]) if rows else None


def run_of_log(path):
    for line in open(path):
        if line.startswith('{"world"'):
            d = json.loads(line)
            best = [e for e in d["epochs"] if e.get("final_best")]
            return {"seed": d["seed"], "lr": d["lr"], "epochs_run": sum(1 for e in d["epochs"] if "epoch" in e),
                    "cv_acc_by_epoch": [round(e["cv_acc"], 2) for e in d["epochs"] if "epoch" in e],
                    "accepted": [e["accepted"] for e in d["epochs"] if "epoch" in e],
                    "best_accepted_cv_acc": round(best[0]["cv_acc"], 3) if best else None,
                    "cv_frames": d["epochs"][0]["cv_frames"], "steps_per_epoch_rank0": d["epochs"][0]["steps_rank0"],
                    "wall_s": d["wall_s"]}
    raise SystemExit(f"{path}: no result line")


def stats(vals):
    return {"mean": round(statistics.mean(vals), 2), "sd": round(statistics.stdev(vals), 2) if len(vals) > 1 else 0.0,
            "min": min(vals), "max": max(vals), "n": len(vals)}


def main():
    r5d, bench_dir = sys.argv[1], sys.argv[2]
    t_ar = float(sys.argv[3]) if len(sys.argv) > 3 else 40.0
    r04 = json.load(open(os.path.join(REPO, "profiles", "r04_dp_accuracy_ex01.json")))
    step = {}
    for b in (128, 256, 512, 1024):
        f = last_json(os.path.join(bench_dir, f"mlp3_fdp_b{b}.json"))
        u = last_json(os.path.join(bench_dir, f"mlp3_b{b}.json"))
        step[b] = {"dp_one_rank_ms": f["ms_per_step"], "fused_ms": u["ms_per_step"], "fused_frames_s": u["value"]}
    one_gpu = step[1024]["fused_frames_s"]
    modes = []

    def add(name, what, bunch, global_bunch, lr, seeds):
        acc = [s["best_accepted_cv_acc"] if "best_accepted_cv_acc" in s else s["final_cv_acc_best_accepted"]
               for s in seeds]
        m = {"mode": name, "what": what, "bunch_per_rank": bunch, "global_bunch": global_bunch, "lr": lr,
             "cv_acc": stats(acc), "seeds": seeds}
        if bunch in step and global_bunch > bunch:
            t = step[bunch]["dp_one_rank_ms"] * 1e3
            m["dp_step_one_rank_us"] = round(t, 1)
            m["n8_frames_s_bound_t_ar0"] = round(8 * bunch / (t * 1e-6))
            m["n8_frames_s_bound_t_ar"] = round(8 * bunch / ((t + t_ar) * 1e-6))
            m["n8_speedup_vs_one_gpu_fused_b1024"] = round(m["n8_frames_s_bound_t_ar"] / one_gpu, 2)
        elif global_bunch == bunch:
            m["frames_s_one_gpu_fused"] = step[bunch]["fused_frames_s"] if bunch in step else None
        modes.append(m)

    R = r04["runs"]
    add("n1", r04["configs"]["ex01_w1"], 1024, 1024, 8.0, R["ex01_w1"]["seeds"])
    add("n8_strong_128", r04["configs"]["ex01_w8strong"], 128, 1024, 8.0, R["ex01_w8strong"]["seeds"])
    rule_text = {"lin": "linear in the global bunch: 8 x {g}/1024", "half": "half the linear rule: 8 x {g}/1024 / 2",
                 "n1": "the N = 1 recipe's lr, unscaled", "n1half": "half the N = 1 recipe's lr"}
    for b, g in ((256, 2048), (512, 4096)):
        for rule in ("lin", "half", "n1", "n1half"):
            logs = sorted(glob.glob(os.path.join(r5d, f"ex01_w8_b{b}_{rule}_s*.log")),
                          key=lambda p: int(re.search(r"_s(\d+)\.log$", p).group(1)))
            if not logs:
                continue
            seeds = [run_of_log(p) for p in logs]
            lr = seeds[0]["lr"]
            add(f"n8_{b}_{rule}", f"N=8, {b} frames per rank (global {g}), lr {lr:g} ({rule_text[rule].format(g=g)}), "
                f"half-epoch linear warm-up, newbob", b, g, lr, seeds)
    add("n8_weak_1024", r04["configs"]["ex01_w8weak"], 1024, 8192, 8.0, R["ex01_w8weak"]["seeds"])
    add("n8_weak_1024_lr4", r04["configs"]["ex01_w8weak_lr4_warm1"], 1024, 8192, 4.0, R["ex01_w8weak_lr4_warm1"]["seeds"])
    base = next(m for m in modes if m["mode"] == "n1")["cv_acc"]
    for m in modes:
        m["cv_acc_gap_vs_n1_mean"] = round(m["cv_acc"]["mean"] - base["mean"], 2)
        m["within_n1_seed_range"] = base["min"] <= m["cv_acc"]["mean"] <= base["max"]
    out = {"what": "examples/01 MLP3 598:1024:135, tools/dp_accuracy.py --corpus ex01 --newbob (start 0.01 / end 0.001), "
                   "--cv-bunch 128 (one 2,816-frame held-out set for every mode), N ranks as processes on one MI355X "
                   "exchanging through the host transport (the RCCL exchange's protocol), 5 seeds; reported: the best "
                   "ACCEPTED epoch's CV frame accuracy",
           "one_rank_dp_step_by_bunch": step, "t_ar_us_assumed": t_ar,
           "projection": "N=8 frames/s <= 8 B / (t_dp(B) + t_ar): t_dp = the one-rank DP step at bunch B measured here; "
                         "t_ar = the 3.24 MB 8-GPU all-reduce, NOT measured (one GPU per call), assumed",
           "one_gpu_fused_b1024_frames_s": one_gpu, "modes": modes}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
