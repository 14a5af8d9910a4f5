#!/usr/bin/env python3
"""Per-step times of the dnn4 SGD step from a cold start: the same trainer as bench.py (440 -> 2048x4 -> 4000,
bunch 1024, synthetic frames), then `steps` single steps each timed on the host with a device synchronize
(the sync adds a few us a step; the trend is what matters), and the GPU's shader clock from in-kernel stamps
where rocm-smi is not readable.  usage: python tools/warmup_trace.py [steps] [idle_ms]
idle_ms: a host sleep after the first 60 steps, then 30 more steps (does an idle gap cost the ramp again?)"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import bench  # noqa: E402
import tnet_amd  # noqa: E402
from tnet_amd import Objective, Trainer  # noqa: E402
from tnet_amd._lib import lib  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
idle_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
dims = [440, 2048, 2048, 2048, 2048, 4000]
B, cache = 1024, 65536
net = bench.build_network(dims)
net.set_learn_rate(0.008)
net.set_grad_div_frm(True)
obj = Objective()
tr = Trainer(net, obj, bunchsize=B, cachesize=cache, seed=123, randomize=True)
X, L = bench.synth_frames(cache, dims[0], dims[-1], seed=1000)
taken = lib().tnet_trainer_prefill(tr.h, X.ctypes.data, X.shape[0], X.shape[1], X.shape[1], L.ctypes.data)
assert taken == cache, taken
tnet_amd.synchronize()


def run(n):
    out = []
    for _ in range(n):
        t0 = time.perf_counter()
        tr.replay(1)
        tnet_amd.synchronize()
        out.append(round(1e3 * (time.perf_counter() - t0), 4))
    return out


cold = run(steps)
time.sleep(idle_ms / 1e3)
after_idle = run(30)
print(json.dumps({"per_step_ms_cold_start": cold, "idle_ms": idle_ms, "per_step_ms_after_idle": after_idle,
                  "note": "host-timed single steps with a synchronize each (a few us of sync overhead a step)"}),
      flush=True)
