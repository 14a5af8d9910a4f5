#!/usr/bin/env python3
"""Diagnostics for test_newbob_scheduler_over_tnetcu_matches_reference: the newbob schedule of
examples/01 (80 / 20 utterances, bunch 960, LEARNRATE 7.68 in CUDA mode) run three ways on the GPU --
  text : the native Trainer, the model handed between epochs as 6-digit .nnet text (Network.write /
         Network(path=...)), as TNetCu does through --TARGETMMF / -H
  mem  : the native Trainer, the model kept in device memory between epochs (no text round trip)
  F    : as text, but GRADDIVFRM=F with the per-frame rate (the CPU-equivalent semantics)
printing per iteration the learning rate, TR / CV err/frm and the decision."""
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import tnet_amd  # noqa: E402
from tnet_amd import formats, newbob  # noqa: E402

EX = os.path.join(REPO, "tests", "golden", "ex01")
c = formats.read_corpus(os.path.join(EX, "test.scp"), os.path.join(EX, "test_3s.mlf"),
                        os.path.join(EX, "mono_state_phn_set_135_phn"))
transform = tnet_amd.Network(path=os.path.join(EX, "Hamm_dct_norm"))
tr_f, tr_l, cv_f, cv_l = c.feats[:80], c.labels[:80], c.feats[80:], c.labels[80:]


def epoch(net, feats, labels, crossval):
    obj = tnet_amd.Objective()
    t = tnet_amd.Trainer(net, obj, bunchsize=960, cachesize=14400, seed=123, randomize=not crossval,
                         crossval=crossval)
    t.set_transform(transform, 25, 25)
    t.train_corpus(feats, labels)
    e, n, _ = obj.stats()
    return "%.6g" % (e / n)


for mode in sys.argv[1:] or ["text", "mem", "F"]:
    with tempfile.TemporaryDirectory() as td:
        init = os.path.join(td, "init.nnet")
        formats.write_nnet(formats.gen_mlp_init([598, 1024, 135], seed=1), init, precision=6)
        gdf = mode != "F"
        nb = newbob.Newbob("7.68", 960, threads=None if gdf else 1, max_iter=6, end_halving_inc=0.01)
        best = tnet_amd.Network(path=init)
        nb.initial(epoch(best, cv_f, cv_l, True))
        best_path, best_params = init, None
        for it in range(1, 7):
            net = tnet_amd.Network(path=best_path if mode != "mem" else init)
            if mode == "mem" and best_params is not None:   # the best network's fp32 weights, no text
                for k, (W, b) in enumerate(best_params):
                    net.set_params(2 * k, W, b)
            net.set_learn_rate(float(nb.lrate) if gdf else float(nb.lrate))
            net.set_grad_div_frm(gdf)
            tr = epoch(net, tr_f, tr_l, False)
            out = os.path.join(td, f"it{it}.nnet")
            net.write(out)
            cv = epoch(net if mode == "mem" else tnet_amd.Network(path=out), cv_f, cv_l, True)
            acc = nb.decide(it, tr, cv, out)
            print(mode, it, nb.history[-1].lrate, tr, cv, acc, flush=True)
            if acc:
                best_path, best_params = out, [(W.copy(), b.copy()) for W, b in net.linear_params()]
            if nb.done:
                break
