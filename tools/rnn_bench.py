#!/usr/bin/env python3
"""BASELINE config 5 (TRecurrentCu: 440 -> 512-unit Elman RNN -> softmax, 1000-frame utterances,
BPTT order 4, frame-by-frame SGD) on the GPU, next to the oracle's C restatement of the same loop on
one host core (oracle/tnet_oracle.c orc_rnn_utterance: the reference's CuRecurrent arithmetic in
plain C -- a CPU stand-in, not the reference binary, which is CUDA-only).

usage: python tools/rnn_bench.py [utterances] [senones]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import oracle as orc  # noqa: E402
import tnet_amd  # noqa: E402
from tnet_amd import Network, Objective, RnnTrainer, formats  # noqa: E402

n_utt = int(sys.argv[1]) if len(sys.argv) > 1 else 4
S = int(sys.argv[2]) if len(sys.argv) > 2 else 135
nIn, H, T, bptt, lr = 440, 512, 1000, 4, 0.01
rng = np.random.default_rng(0)
layers = formats.gen_recurrent_init(nIn, H, S, seed=7)
feats = [rng.standard_normal((T, nIn)).astype(np.float32) for _ in range(n_utt)]
labels = [rng.integers(0, S, T).astype(np.int32) for _ in range(n_utt)]

net = Network.from_layers(layers)
net.set_learn_rate(lr)
obj = Objective()
tr = RnnTrainer(net, obj, bptt=bptt)
tr.train_utterance(feats[0][:50], labels[0][:50])  # warm-up
tnet_amd.synchronize()
rates = []
for rep in range(3):  # three passes over the utterances: the median (single-frame launches jitter)
    t0 = time.perf_counter()
    tr.train_corpus(feats, labels)
    tnet_amd.synchronize()
    rates.append(n_utt * T / (time.perf_counter() - t0))
gpu = float(np.median(rates))

m = orc.RNN(layers[0].W, layers[0].b, layers[1].W, layers[1].b)
t0 = time.perf_counter()
m.utterance(feats[0], labels[0], bptt, lr, 0.0, 0.0)
cpu = T / (time.perf_counter() - t0)
# per-frame HBM bound (the weights are updated every frame, so every frame streams them): recurrent
# forward reads Wr [(nIn+H) x H]; the output layer reads W2 [H x S] once for z and once more + writes it
# for the fused backprop/update; the BPTT GEMVs read the recurrent block [H x H] bptt times; the
# recurrent update reads and writes Wr
wr, w2, hh = 4.0 * (nIn + H) * H, 4.0 * H * S, 4.0 * H * H
bytes_frame = wr + w2 + 2 * w2 + bptt * hh + 2 * wr
bound = 8000e9 / bytes_frame
print(json.dumps({"config": f"TRecurrentCu RNN {nIn}->{H} (BPTT {bptt})->{S}, {T}-frame utterances",
                  "gpu_frames_per_s": round(gpu, 1),
                  "roofline": {"bound": "hbm", "achieved": round(gpu * bytes_frame / 1e9, 1), "peak": 8000.0,
                               "unit": "GB/s", "frac": round(gpu / bound, 4),
                               "algorithmic_bytes_per_frame": bytes_frame,
                               "basis": "per-frame weight streaming (Wr fwd + W2 fwd + W2 read/write in the fused "
                                        "backprop/update + bptt x recurrent block + Wr read/write)"},
                  "cpu_frames_per_s": round(cpu, 1), "cpu": "oracle C restatement orc_rnn_utterance, 1 core"}),
      flush=True)
print(f"RNN {nIn}->{H}(recurrent, bptt {bptt})->{S}, {T}-frame utterances: GPU {gpu:.0f} frames/s (median of "
      f"{', '.join(f'{r:.0f}' for r in rates)}), oracle C restatement (1 core) {cpu:.0f} frames/s", flush=True)
