#!/usr/bin/env python3
"""Chaos check on the oracle: epoch 1 of the examples/01 newbob schedule (GRADDIVFRM=T) with one init weight
moved by one ulp (k > 0); usage: oracle_perturb.py k0 k1 (profiles/r03_ex01_newbob_variants.txt)"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd")); sys.path.insert(0, os.path.join(REPO, "oracle")); os.chdir(REPO)
import numpy as np, oracle as orc
from tnet_amd import formats
c=formats.read_corpus('tests/golden/ex01/test.scp','tests/golden/ex01/test_3s.mlf','tests/golden/ex01/mono_state_phn_set_135_phn')
L=formats.read_nnet('tests/golden/ex01/Hamm_dct_norm')
X=np.concatenate([orc.frontend_forward(L,x,25,25) for x in c.feats[:80]]); Y=np.concatenate(c.labels[:80])
sched=orc.epoch_schedule([len(l) for l in c.labels[:80]], 14400, 960, 123)
layers=formats.round_trip_text(formats.gen_mlp_init([598,1024,135],seed=1),6)
for k in range(int(sys.argv[1]), int(sys.argv[2])):
    net=orc.MLP.from_layers(layers)
    if k>0:
        r=np.random.default_rng(k); i=r.integers(0,598); j=r.integers(0,1024)
        net.W[0][i,j]=np.nextafter(net.W[0][i,j], np.float32(1))   # one ulp in one weight
    for b in sched: net.step(X[b],Y[b],7.68,graddivfrm=True)
    print(k, net.xent/net.frames, 100*net.correct/net.frames, flush=True)
