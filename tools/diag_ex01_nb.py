#!/usr/bin/env python3
"""Diagnostics: newbob iteration 1 of tests/test_ex01.py (80 examples/01 utterances, bunch 960,
CUDA-mode lr 7.68 with GRADDIVFRM=T) through the native trainer and the drop-in driver, seeded on the
command line and through an STK config file."""
import os, re, subprocess, sys, tempfile
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import numpy as np
import tnet_amd
from tnet_amd import formats
EX = os.path.join(REPO, "tests", "golden", "ex01")
f = dict(scp=os.path.join(EX, "test.scp"), mlf=os.path.join(EX, "test_3s.mlf"),
         states=os.path.join(EX, "mono_state_phn_set_135_phn"), transform=os.path.join(EX, "Hamm_dct_norm"))
c = formats.read_corpus(f["scp"], f["mlf"], f["states"])
for gdf, lr in ((True, 7.68), (False, 0.008)):
    net = tnet_amd.Network.from_layers(formats.round_trip_text(formats.gen_mlp_init([598, 1024, 135], seed=1), 6))
    net.set_learn_rate(lr)
    net.set_grad_div_frm(gdf)
    obj = tnet_amd.Objective()
    tr = tnet_amd.Trainer(net, obj, bunchsize=960, cachesize=14400, seed=123)
    tr.set_transform(tnet_amd.Network(path=f["transform"]), 25, 25)
    tr.train_corpus(c.feats[:80], c.labels[:80])
    e, n, k = obj.stats()
    print(f"native gdf={gdf} lr={lr}: err/frm {e / n:.6f} frames {n} acc {100 * k / n:.4f}", flush=True)
lines = [l for l in open(f["scp"]) if l.strip()]
drv = os.path.join(REPO, "oracle", "_ref", "TNetCu_amd")
with tempfile.TemporaryDirectory() as td:
    tr_scp = os.path.join(td, "train.scp")
    open(tr_scp, "w").writelines(os.path.join(EX, l.strip()) + "\n" for l in lines[:80])
    init = os.path.join(td, "mlp.init")
    formats.write_nnet(formats.gen_mlp_init([598, 1024, 135], seed=1), init, precision=6)
    conf = os.path.join(td, "tnet.conf")
    open(conf, "w").write("SEED = 123\n")
    base = [drv, "-H", init, "-I", f["mlf"], "-L", "*/", "-X", "lab", "-S", tr_scp, "--BUNCHSIZE=960",
            "--CACHESIZE=14400", f"--OUTPUTLABELMAP={f['states']}", "--STARTFRMEXT=25", "--ENDFRMEXT=25",
            f"--FEATURETRANSFORM={f['transform']}", f"--TARGETMMF={os.path.join(td, 'o.nnet')}", "--RANDOMIZE=TRUE"]
    for extra in (["--LEARNINGRATE=7.68", "--SEED=123"], ["--LEARNINGRATE=7.68", "-C", conf],
                  ["--LEARNINGRATE=0.008", "--GRADDIVFRM=FALSE", "--SEED=123"]):
        p = subprocess.run(base + extra, capture_output=True, text=True, cwd=td)
        m = re.findall(r"Xent:.*", p.stdout)
        print("drop-in", " ".join(extra), m[-1:] if m else p.stdout[-800:] + p.stderr[-800:], flush=True)
