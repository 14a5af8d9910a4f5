#!/usr/bin/env python3
"""One-step errors along the REFERENCE trajectory of examples/01's run_test.CPU.sh epoch (57 bunches of 960,
lr 0.008, GRADDIVFRM=F): oracle/_ref/ref_harness trajectory gives the reference TNetLib parameters before
every step; at each step the GPU network is reset to them, trains the bunch once, and its output / update
are compared with the reference's -- and, for the bias updates, with the fp64 oracle step from the same
parameters (the reference sums a bias gradient column in a float loop over 960 rows: its own rounding).
Prints one line per step.  usage: diag_step_resync.py [steps]"""
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
import numpy as np  # noqa: E402

import make_ex01 as mk  # noqa: E402
import oracle as orc  # noqa: E402
import tnet_amd  # noqa: E402
from tnet_amd import formats  # noqa: E402

nsteps = int(sys.argv[1]) if len(sys.argv) > 1 else None


def rel(got, new, old):
    d = new.astype(np.float64) - old
    return np.linalg.norm(got.astype(np.float64) - new) / max(np.linalg.norm(d), 1e-30)


with tempfile.TemporaryDirectory() as td:
    params, Yr, X, L, cfg = mk.trajectory_run(td, nsteps)
B, lr = cfg["bunch"], cfg["lr"]
net = tnet_amd.Network.from_layers(formats.round_trip_text(formats.gen_mlp_init(mk.INIT["dims"], seed=1), 6))
net.set_learn_rate(lr)
net.set_grad_div_frm(False)
net.keep_output(True)
print("step  Y rel    | gpu-ref: W0 b0 W1 b1 | orc(float b loop)-ref: b0 b1, orc64-ref: b0 b1 | gpu-orc64: W0 b0 W1 b1")
for s in range(len(Yr)):
    before, after = mk.split_params(params[s]), mk.split_params(params[s + 1])
    for k, (W, b) in enumerate(before):
        net.set_params(2 * k, W, b)
    obj = tnet_amd.Objective()
    Xs, Ls = X[s * B:(s + 1) * B], L[s * B:(s + 1) * B]
    net.train_bunch(obj, tnet_amd.DeviceArray.from_numpy(Xs), tnet_amd.DeviceArray.vector(Ls))
    Yg = net.output(3, B)
    ref = orc.MLP([w for w, _ in before], [b for _, b in before])   # fp64-accumulated update (GPU semantics)
    ref.step(Xs, Ls, lr, graddivfrm=False)
    fl = orc.MLP([w for w, _ in before], [b for _, b in before])    # the reference's float bias loop
    fl.step(Xs, Ls, lr, graddivfrm=False, cpu_semantics=True)
    gp = net.linear_params()
    yerr = np.linalg.norm(Yg.astype(np.float64) - Yr[s]) / np.linalg.norm(Yr[s].astype(np.float64))
    gr = [rel(gp[k][j], after[k][j], before[k][j]) for k in range(2) for j in range(2)]
    orr = [rel(fl.b[k], after[k][1], before[k][1]) for k in range(2)] + \
          [rel(ref.b[k], after[k][1], before[k][1]) for k in range(2)]
    go = [rel(gp[k][j], (ref.W, ref.b)[j][k], before[k][j]) for k in range(2) for j in range(2)]
    print(f"{s:4d}  {yerr:.2e} | " + " ".join(f"{e:.2e}" for e in gr) + " | " + " ".join(f"{e:.2e}" for e in orr) +
          " | " + " ".join(f"{e:.2e}" for e in go), flush=True)
