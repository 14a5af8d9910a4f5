#!/usr/bin/env python3
"""Phase timing of the persistent RNN utterance kernel (rnn_persistent.hip) from in-kernel
s_memrealtime stamps of workgroup 0 (diagnostic; tnet_rnn_utterance_stamps).

usage: python tools/rnn_stamps.py [senones]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import numpy as np  # noqa: E402

import tnet_amd  # noqa: E402
from tnet_amd import DeviceArray, Network, Objective, RnnTrainer, formats  # noqa: E402
from tnet_amd._lib import check, lib  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 135
nIn, H, T = 440, 512, 1000
rng = np.random.default_rng(0)
net = Network.from_layers(formats.gen_recurrent_init(nIn, H, S, seed=7))
net.set_learn_rate(0.01)
tr = RnnTrainer(net, Objective(), bptt=4)
x = rng.standard_normal((T, nIn)).astype(np.float32)
l = rng.integers(0, S, T).astype(np.int32)
tr.train_utterance(x, l)  # warm-up
buf = DeviceArray(T, 8, np.int64, stride=8)
check(lib().tnet_rnn_utterance_stamps(buf.ptr))
tr.train_utterance(x, l)
tnet_amd.synchronize()
check(lib().tnet_rnn_utterance_stamps(None))
st = buf.numpy().astype(np.float64) / 100.0  # us
names = ["fwd rec", "AG1 wait", "out logits", "AG2 wait+norm", "bwd out + RS", "BPTT (RS waits)", "W update"]
d = np.diff(st[:, :8], axis=1)[10:]
frame = np.diff(st[:, 0])[10:]
print(f"senones {S}: frame {frame.mean():.2f} us ({1e6 / frame.mean():.0f} frames/s in-kernel)")
for k, n in enumerate(names):
    print(f"  {n:18s} {d[:, k].mean():7.2f} us")
