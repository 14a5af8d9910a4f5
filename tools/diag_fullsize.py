#!/usr/bin/env python3
"""Diagnostics for tests/test_gpu_fullsize.py: per-layer update errors of the fused TrainBunch path
vs the oracle, and where in W they sit (rows / columns / tiles).  usage: diag_fullsize.py [dims...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import oracle as orc  # noqa: E402
from tnet_amd import DeviceArray, Network, Objective, formats  # noqa: E402

dims = [int(a) for a in sys.argv[1:]] or [440, 2048, 2048, 4000]
steps = int(os.environ.get("STEPS", "1"))
B, lr = int(os.environ.get("BUNCH", "1024")), 1.0
layers = formats.gen_mlp_init(dims, seed=2)
net = Network.from_layers(layers)
net.set_learn_rate(lr)
net.set_grad_div_frm(True)
obj = Objective()
ref = orc.MLP.from_layers(layers)
W0 = [w.astype(np.float64) for w in ref.W]
b0 = [b.astype(np.float64) for b in ref.b]
rng = np.random.default_rng(7)
for s in range(steps):
    X = rng.standard_normal((B, dims[0])).astype(np.float32)
    L = rng.integers(0, dims[-1], B).astype(np.int32)
    net.train_bunch(obj, DeviceArray.from_numpy(X), DeviceArray.vector(L))
    ref.step(X, L, lr)
for k, (W, b) in enumerate(net.linear_params()):
    dr = ref.W[k].astype(np.float64) - W0[k]
    dg = W.astype(np.float64) - W0[k]
    e = dg - dr
    rel = np.linalg.norm(e) / np.linalg.norm(dr)
    rowe = np.linalg.norm(e, axis=1) / np.maximum(np.linalg.norm(dr, axis=1), 1e-30)
    cole = np.linalg.norm(e, axis=0) / np.maximum(np.linalg.norm(dr, axis=0), 1e-30)
    bre = np.linalg.norm((b.astype(np.float64) - b0[k]) - (ref.b[k] - b0[k])) / np.linalg.norm(ref.b[k] - b0[k])
    print(f"layer {k} {W.shape}: dW rel {rel:.3e}  db rel {bre:.3e}  |dW| {np.abs(dr).max():.3e}  |W| {np.abs(W0[k]).max():.3e}")
    bad_r = np.argsort(rowe)[-5:][::-1]
    bad_c = np.argsort(cole)[-5:][::-1]
    print("   worst rows", [(int(i), f"{rowe[i]:.2e}") for i in bad_r], " median row", f"{np.median(rowe):.2e}")
    print("   worst cols", [(int(i), f"{cole[i]:.2e}") for i in bad_c], " median col", f"{np.median(cole):.2e}")
    # ulp-level floor of the fp32 weights themselves: |W| eps vs |dW|
    print(f"   fp32 storage floor of W (eps*|W| / |dW|, Frobenius): "
          f"{np.linalg.norm(np.float32(2**-24) * np.abs(W0[k])) / np.linalg.norm(dr):.3e}")
