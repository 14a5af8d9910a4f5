#!/usr/bin/env python3
"""Is the GPU's departure from the reference on examples/01 rounding chaos or a systematic error?

Trains the first epoch of the scheduler test's 80 utterances (bunch 960, reference cache order) step
by step on the GPU (fused TrainBunch) and in the oracle (fp64-accumulated restatement) with the same
semantics, and prints per step the relative distance of the weights, next to the distance between
two oracle runs whose ONLY difference is the rounding of the update (CPU semantics lr 0.008 with
summed gradients vs GPU semantics GRADDIVFRM=T lr 7.68 / 960): chaos shows the same exponential
growth in both columns from ~1e-7; a systematic error would jump above the oracle-vs-oracle column.
usage: diag_chaos.py [steps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import oracle as orc  # noqa: E402
from tnet_amd import formats  # noqa: E402

nsteps = int(sys.argv[1]) if len(sys.argv) > 1 else 48
gpu = os.environ.get("NO_GPU") != "1"
EX = os.path.join(REPO, "tests", "golden", "ex01")
c = formats.read_corpus(os.path.join(EX, "test.scp"), os.path.join(EX, "test_3s.mlf"),
                        os.path.join(EX, "mono_state_phn_set_135_phn"))
L = formats.read_nnet(os.path.join(EX, "Hamm_dct_norm"))
feats, labs = c.feats[:80], c.labels[:80]
X = np.concatenate([orc.frontend_forward(L, x, 25, 25) for x in feats])
Y = np.concatenate(labs)
sched = orc.epoch_schedule([len(l) for l in labs], 14400, 960, 123)[:nsteps]
layers = formats.round_trip_text(formats.gen_mlp_init([598, 1024, 135], seed=1), 6)
W0 = [L_.W.astype(np.float64) for L_ in layers if L_.W is not None]


def dist(Wa, Wb):
    num = sum(np.linalg.norm(np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2 for a, b in zip(Wa, Wb))
    den = sum(np.linalg.norm(np.asarray(b, np.float64) - w0) ** 2 for b, w0 in zip(Wb, W0))
    return np.sqrt(num / den)


o_t = orc.MLP.from_layers(layers)
o_c = orc.MLP.from_layers(layers)
o_f = orc.MLP.from_layers(layers)
if gpu:
    import tnet_amd
    nets = {}
    for mode in ("T", "F"):
        n = tnet_amd.Network.from_layers(layers)
        n.set_learn_rate(7.68 if mode == "T" else 0.008)
        n.set_grad_div_frm(mode == "T")
        nets[mode] = (n, tnet_amd.Objective())
print("step  orcT-vs-orcCPU  orcF-vs-orcCPU  gpuT-vs-orcT  gpuF-vs-orcF  gpuT-vs-gpuF")
for s, b in enumerate(sched):
    o_t.step(X[b], Y[b], 7.68, graddivfrm=True)
    o_c.step(X[b], Y[b], 0.008, cpu_semantics=True)
    o_f.step(X[b], Y[b], 0.008, graddivfrm=False)
    row = f"{s:4d}  {dist(o_t.W, o_c.W):.3e}       {dist(o_f.W, o_c.W):.3e}"
    if gpu:
        Wg = {}
        for mode, (n, obj) in nets.items():
            n.train_bunch(obj, tnet_amd.DeviceArray.from_numpy(np.ascontiguousarray(X[b])),
                          tnet_amd.DeviceArray.vector(Y[b].astype(np.int32)))
            Wg[mode] = [w for w, _ in n.linear_params()]
        row += f"     {dist(Wg['T'], o_t.W):.3e}     {dist(Wg['F'], o_f.W):.3e}     {dist(Wg['T'], Wg['F']):.3e}"
    print(row, flush=True)
print("oracle err/frm T / CPU / F:", o_t.xent / o_t.frames, o_c.xent / o_c.frames, o_f.xent / o_f.frames)
if gpu:
    for mode, (n, obj) in nets.items():
        e, fr, k = obj.stats()
        print(f"gpu {mode}: err/frm {e / fr:.6f}")
