#!/usr/bin/env python3
"""Where an RNN frame's time goes (BASELINE config 5: 440 -> 512 recurrent, BPTT 4 -> 135 / 4000 senones).

  run S          train two 1000-frame utterances on the fused frame chain (graph replay on, as in
                 tools/rnn_bench.py) -- meant to run under `rocprofv3 --kernel-trace`
  summarize CSV  read the kernel trace (rocprofv3's *_kernel_trace.csv) of the LAST utterance: the frame period,
                 per kernel kind its mean duration and the mean idle gap before it (the dependent-launch cost),
                 printed as one JSON object

usage: python tools/rnn_frame_trace.py run 135
       python tools/rnn_frame_trace.py summarize gpurun_out/.../run_kernel_trace.csv"""
import csv
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(S):
    sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
    import numpy as np

    import tnet_amd
    from tnet_amd import Network, Objective, RnnTrainer, formats

    nIn, H, T, bptt, lr = 440, 512, 1000, 4, 0.01
    rng = np.random.default_rng(0)
    net = Network.from_layers(formats.gen_recurrent_init(nIn, H, S, seed=7))
    net.set_learn_rate(lr)
    tr = RnnTrainer(net, Objective(), bptt=bptt)
    feats = [rng.standard_normal((T, nIn)).astype(np.float32) for _ in range(3)]
    labels = [rng.integers(0, S, T).astype(np.int32) for _ in range(3)]
    for f, l in zip(feats, labels):  # 1st: eager, 2nd: recorded + replayed, 3rd: replayed (the one summarized)
        tr.train_utterance(f, l)
    tnet_amd.synchronize()
    print(json.dumps({"senones": S, "utterances": 3, "frames": T}), flush=True)


def short(name):
    n = name.split("(")[0]
    for k in ("rnn_out_full", "rnn_out_bwd", "gemv_rows", "rnn_update", "rowvec", "argmax_correct", "rnn_"):
        if k in n:
            return n.replace("void ", "").replace("tnetk::", "")
    return n.replace("void ", "").replace("tnetk::", "")


def summarize(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # the last utterance: the kernels after the last-but-one argmax_correct launch (one per utterance, at its end)
    ends = [i for i, r in enumerate(rows) if "argmax_correct" in r[2]]
    if len(ends) < 2:
        raise SystemExit("fewer than two utterances in the trace")
    seg = rows[ends[-2] + 1:ends[-1]]
    T = 1000
    span = seg[-1][1] - seg[0][0]
    per = defaultdict(lambda: [0, 0.0, 0.0])  # count, busy ns, gap-before ns
    busy = 0
    for i, (s, e, n) in enumerate(seg):
        k = short(n)
        per[k][0] += 1
        per[k][1] += e - s
        busy += e - s
        if i:
            per[k][2] += max(0, s - seg[i - 1][1])
    out = {"trace": os.path.basename(path), "frames": T, "launches": len(seg),
           "launches_per_frame": round(len(seg) / T, 2), "frame_us": round(span / T / 1e3, 3),
           "busy_us_per_frame": round(busy / T / 1e3, 3), "idle_us_per_frame": round((span - busy) / T / 1e3, 3),
           "kernels": {k: {"per_frame": round(c / T, 2), "mean_us": round(b / c / 1e3, 3),
                           "mean_gap_before_us": round(g / c / 1e3, 3)} for k, (c, b, g) in
                       sorted(per.items(), key=lambda kv: -kv[1][1])}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) >= 3 and sys.argv[1] == "run":
        run(int(sys.argv[2]))
    elif len(sys.argv) >= 3 and sys.argv[1] == "summarize":
        summarize(sys.argv[2])
    else:
        raise SystemExit(__doc__)
