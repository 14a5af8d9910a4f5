#!/usr/bin/env python3
"""One-step errors along the oracle's trajectory: at every step of examples/01's newbob epoch 1
(80 utterances, bunch 960, GRADDIVFRM=T lr 7.68) the GPU network is reset to the oracle's weights, runs
the same bunch through the fused TrainBunch, and its outputs / update are compared with the oracle's
step -- a per-step arithmetic anomaly (not chaos) shows as a step whose error jumps above the ~1e-6
rounding level.  usage: diag_step_resync.py [steps] [lr] [gdf]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import oracle as orc  # noqa: E402
import tnet_amd  # noqa: E402
from tnet_amd import formats  # noqa: E402

nsteps = int(sys.argv[1]) if len(sys.argv) > 1 else 48
lr = float(sys.argv[2]) if len(sys.argv) > 2 else 7.68
gdf = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
EX = os.path.join(REPO, "tests", "golden", "ex01")
c = formats.read_corpus(os.path.join(EX, "test.scp"), os.path.join(EX, "test_3s.mlf"),
                        os.path.join(EX, "mono_state_phn_set_135_phn"))
L = formats.read_nnet(os.path.join(EX, "Hamm_dct_norm"))
X = np.concatenate([orc.frontend_forward(L, x, 25, 25) for x in c.feats[:80]])
Y = np.concatenate(c.labels[:80])
sched = orc.epoch_schedule([len(l) for l in c.labels[:80]], 14400, 960, 123)[:nsteps]
layers = formats.round_trip_text(formats.gen_mlp_init([598, 1024, 135], seed=1), 6)
ref = orc.MLP.from_layers(layers)
net = tnet_amd.Network.from_layers(layers)
net.set_learn_rate(lr)
net.set_grad_div_frm(gdf)
net.keep_output(True)
print("step  dW0 rel   dW1 rel   db0 rel   db1 rel   max|dY|    xent(gpu-orc)/orc  y_min      hid_sat")
for s, b in enumerate(sched):
    before = [(w.copy(), bb.copy()) for w, bb in zip(ref.W, ref.b)]
    for k, (w, bb) in enumerate(before):
        net.set_params(2 * k, w, bb)
    obj = tnet_amd.Objective()
    net.train_bunch(obj, tnet_amd.DeviceArray.from_numpy(np.ascontiguousarray(X[b])),
                    tnet_amd.DeviceArray.vector(Y[b].astype(np.int32)))
    x0 = ref.xent
    Yr, _ = ref.step(X[b], Y[b], lr, graddivfrm=gdf)
    Yg = net.output(3, len(b))
    hid = net.output(1, len(b))
    errs = []
    for k, (Wg, bg) in enumerate(net.linear_params()):
        for got, want, old in ((Wg, ref.W[k], before[k][0]), (bg, ref.b[k], before[k][1])):
            d = want.astype(np.float64) - old
            errs.append(np.linalg.norm(got.astype(np.float64) - want) / max(np.linalg.norm(d), 1e-30))
    e, f, _ = obj.stats()
    xr = ref.xent - x0
    print(f"{s:4d}  {errs[0]:.2e}  {errs[2]:.2e}  {errs[1]:.2e}  {errs[3]:.2e}  {np.abs(Yg - Yr).max():.2e}  "
          f"{(e - xr) / xr:+.2e}  {Yr.min():.2e}  {np.mean((hid < 1e-6) | (hid > 1 - 1e-6)):.3f}", flush=True)
