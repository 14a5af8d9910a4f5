#!/usr/bin/env python3
"""Does the native Trainer's data path (host intake -> GPU transform -> frame trim -> cache -> lrand48
shuffle -> bunches) feed the same bunches as the reference's order?  Trains examples/01's first cache
fill (bunch 960, cache 14400 = 15 bunches, GRADDIVFRM=F lr 0.008) through tnet_amd.Trainer and the same
steps through the oracle on the oracle's schedule, and prints the weight distance -- rounding level
(~1e-6) if the bunches agree, O(1e-1) if any frame or label differs."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import oracle as orc  # noqa: E402
import tnet_amd  # noqa: E402
from tnet_amd import formats  # noqa: E402

EX = os.path.join(REPO, "tests", "golden", "ex01")
c = formats.read_corpus(os.path.join(EX, "test.scp"), os.path.join(EX, "test_3s.mlf"),
                        os.path.join(EX, "mono_state_phn_set_135_phn"))
L = formats.read_nnet(os.path.join(EX, "Hamm_dct_norm"))
feats, labs = c.feats[:80], c.labels[:80]
layers = formats.round_trip_text(formats.gen_mlp_init([598, 1024, 135], seed=1), 6)
W0 = [l.W.astype(np.float64) for l in layers if l.W is not None]
for xform in ("gpu", "host"):
    net = tnet_amd.Network.from_layers(layers)
    net.set_learn_rate(0.008)
    net.set_grad_div_frm(False)
    obj = tnet_amd.Objective()
    tr = tnet_amd.Trainer(net, obj, bunchsize=960, cachesize=14400, seed=123)
    if xform == "gpu":
        tr.set_transform(tnet_amd.Network(path=os.path.join(EX, "Hamm_dct_norm")), 25, 25)
    n = 0
    for x, y in zip(feats, labs):
        tr.add_utterance(x if xform == "gpu" else orc.frontend_forward(L, x, 25, 25), y)
        n += 1
        if tr.steps > 0:
            break
    steps = tr.steps
    X = np.concatenate([orc.frontend_forward(L, x, 25, 25) for x in feats])
    Y = np.concatenate(labs)
    sched = orc.epoch_schedule([len(l) for l in labs], 14400, 960, 123)[:steps]
    ref = orc.MLP.from_layers(layers)
    for b in sched:
        ref.step(X[b], Y[b], 0.008, graddivfrm=False)
    Wg = [w for w, _ in net.linear_params()]
    num = sum(np.linalg.norm(a.astype(np.float64) - b) ** 2 for a, b in zip(Wg, ref.W))
    den = sum(np.linalg.norm(b.astype(np.float64) - w0) ** 2 for b, w0 in zip(ref.W, W0))
    e, f, k = obj.stats()
    print(f"transform on {xform}: {n} utterances in, {steps} steps; weight distance {np.sqrt(num / den):.3e}; "
          f"xent/frm GPU {e / f:.6f} oracle {ref.xent / ref.frames:.6f}; frames {f} / {ref.frames}", flush=True)
