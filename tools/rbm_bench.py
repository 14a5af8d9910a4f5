#!/usr/bin/env python3
"""BASELINE config 4 (TRbmCu: Gauss-Bernoulli RBM 440 -> 2048, CD-1, momentum 0.5, weight cost
0.0002, the driver defaults of src/TRbmCu.cc:169-175) on the GPU, next to the oracle's C
restatement of the same CD-1 step on one host core (oracle/tnet_oracle.c orc_rbm_step: CuRbm's
arithmetic in plain C -- a CPU stand-in; the reference's RBM trainer is CUDA-only, TNetLib has no
CPU RBM).

One step = one bunch through CuRbm: positive phase, HybridTaus binarisation, reconstruction,
negative phase, CD-1 update of W / both biases, and the reconstruction MSE (TRbmCu.cc:329-350).
Frames are synthetic N(0,1) 440-dim rows resident in the GPU cache (the prefill is not timed).
Work per frame: 5 GEMM-equivalents of 440 x 2048 MACs (pos, recon, neg, and the two statistics
products stacked in one update GEMM) = 10 * 440 * 2048 = 9.01 MFLOP.

usage: python tools/rbm_bench.py [bunch] [steps] [cpu_steps]"""
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
from tnet_amd import Network, RbmTrainer, formats  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
cpu_steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
V, H = 440, 2048
lr, mmt, wc = 0.10, 0.50, 0.0002
cache = max(12800 // B, 1) * B
flop_per_frame = 10.0 * V * H

layers = formats.gen_rbm_init(V, H, seed=5)
rng = np.random.default_rng(0)
X = rng.standard_normal((cache, V)).astype(np.float32)

net = Network.from_layers(layers)
tr = RbmTrainer(net, bunchsize=B, cachesize=cache, seed=11, learn_rate=lr, momentum=mmt, weightcost=wc)
taken = tr.prefill(X)
assert taken == cache, taken
tr.replay(50)  # warm-up
tnet_amd.synchronize()
t0 = time.perf_counter()
tr.replay(steps)
tnet_amd.synchronize()
dt = time.perf_counter() - t0
gpu = steps * B / dt

ref = orc.RBM.from_layer(layers[0])
rand = orc.RandState(11, B, H)
t0 = time.perf_counter()
for s in range(cpu_steps):
    ref.step(X[(s * B) % cache:(s * B) % cache + B], rand, lr, mmt, wc)
cpu = cpu_steps * B / (time.perf_counter() - t0)
print(json.dumps({"config": f"TRbmCu Gauss-Bernoulli RBM {V}->{H}, CD-1, bunch {B}", "steps": steps,
                  "gpu_frames_per_s": round(gpu, 1), "ms_per_step": round(1e3 * dt / steps, 4),
                  "gpu_tflops": round(gpu * flop_per_frame / 1e12, 2),
                  "roofline": {"bound": "mfma", "achieved": round(gpu * flop_per_frame / 1e12, 2), "peak": 157.3,
                               "unit": "TFLOP/s", "frac": round(gpu * flop_per_frame / 1e12 / 157.3, 4),
                               "basis": "whole CD-1 step: 10 * 440 * 2048 flop/frame (pos, recon, neg, stacked "
                                        "statistics) / step time, dense fp32 MFMA peak"},
                  "cpu_frames_per_s": round(cpu, 1),
                  "cpu": f"oracle C restatement orc_rbm_step, 1 core, {cpu_steps} steps"}), flush=True)
