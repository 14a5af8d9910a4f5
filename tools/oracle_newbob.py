#!/usr/bin/env python3
"""The newbob schedule of tests/test_ex01.py (examples/01: 80 / 20 utterances, bunch 960, LEARNRATE 7.68,
END_HALVING_INC 0.01, SEED 123) on the ORACLE (fp64-accumulated restatement) with a 6-digit text round trip
between epochs -- CPU semantics (rate / BUNCHSIZE, summed gradients) or GRADDIVFRM=T.  Test infrastructure
(profiles/r03_ex01_newbob_variants.txt).  usage: oracle_newbob.py cpu|gdfT"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd")); sys.path.insert(0, os.path.join(REPO, "oracle")); os.chdir(REPO)
import numpy as np, oracle as orc
from tnet_amd import formats, newbob
c=formats.read_corpus('tests/golden/ex01/test.scp','tests/golden/ex01/test_3s.mlf','tests/golden/ex01/mono_state_phn_set_135_phn')
L=formats.read_nnet('tests/golden/ex01/Hamm_dct_norm')
T=[orc.frontend_forward(L,x,25,25) for x in c.feats]
Xtr=np.concatenate(T[:80]); Ytr=np.concatenate(c.labels[:80]); Xcv=np.concatenate(T[80:]); Ycv=np.concatenate(c.labels[80:])
sched=orc.epoch_schedule([len(l) for l in c.labels[:80]], 14400, 960, 123)
cvs=orc.epoch_schedule([len(l) for l in c.labels[80:]], 14400, 960, 123, randomize=False)
mode=sys.argv[1]
def cv(m):
    net=orc.MLP([w.copy() for w in m.W],[b.copy() for b in m.b])
    Y=net.forward(Xcv[cvs.reshape(-1)]); lab=Ycv[cvs.reshape(-1)]
    _,xe,cor=orc.xent_eval(Y,lab); return xe/len(lab)
layers=formats.round_trip_text(formats.gen_mlp_init([598,1024,135],seed=1),6)
def rt(m):  # 6-digit text round trip between epochs
    lay=[formats.Layer("<biasedlinearity>",w.shape[1],w.shape[0],w,b) for w,b in zip(m.W,m.b)]
    lay2=formats.round_trip_text(lay,6); return orc.MLP([l.W for l in lay2],[l.b for l in lay2])
best=orc.MLP.from_layers(layers)
nb=newbob.Newbob("7.68",960,threads=(1 if mode=='cpu' else None),max_iter=6,end_halving_inc=0.01)
nb.initial("%.6g"%cv(best))
print(mode,'init cv',nb.xent_best,flush=True)
for it in range(1,7):
    m=orc.MLP([w.copy() for w in best.W],[b.copy() for b in best.b])
    lr=float(nb.lrate)
    for b in sched:
        if mode=='cpu': m.step(Xtr[b],Ytr[b],lr,cpu_semantics=True)
        else: m.step(Xtr[b],Ytr[b],lr,graddivfrm=True)
    tr=m.xent/m.frames; m=rt(m); cvx=cv(m)
    acc=nb.decide(it,"%.6g"%tr,"%.6g"%cvx,"x")
    print(mode,it,nb.history[-1].lrate,"%.6g"%tr,"%.6g"%cvx,acc,flush=True)
    if acc: best=m
    if nb.done: break
