#!/usr/bin/env python3
"""Training throughput with the data streamed from host memory (the TNetCu epoch loop), next to the
bench's HBM-resident number: utterances of synthetic 440-dim frames (lengths uniform in [200, 1500],
SURVEY.md 8(d)) are handed to Trainer.add_utterance one by one; the cache (16384 frames, bunch 1024,
shuffled) fills over the copy stream while the previous fill trains (CuCache double buffer).

usage: python tools/intake_bench.py [frames] [cachesize]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import tnet_amd  # noqa: E402
from tnet_amd import Objective, Trainer  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 400000
cache = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
dims = bench.CONFIGS["dnn4"]
rng = np.random.default_rng(0)
lens = []
while sum(lens) < frames:
    lens.append(int(rng.integers(200, 1501)))
X = rng.standard_normal((sum(lens), dims[0]), dtype=np.float32)
L = rng.integers(0, dims[-1], sum(lens)).astype(np.int32)
offs = np.concatenate([[0], np.cumsum(lens)])
utts = [(X[offs[i]:offs[i + 1]], L[offs[i]:offs[i + 1]]) for i in range(len(lens))]


def run(n_utts):
    net = bench.build_network(dims)
    net.set_learn_rate(1.0)
    net.set_grad_div_frm(True)
    obj = Objective()
    tr = Trainer(net, obj, bunchsize=1024, cachesize=cache, seed=123, randomize=True)
    tnet_amd.synchronize()
    t0 = time.perf_counter()
    for x, lab in utts[:n_utts]:
        tr.add_utterance(x, lab)
    tr.finish()
    tnet_amd.synchronize()
    dt = time.perf_counter() - t0
    return tr.steps * 1024, dt


run(20)  # warm-up (allocations, code objects)
trained, dt = run(len(utts))
print(f"streamed from host: {len(utts)} utterances, {sum(lens)} frames, {trained} trained in {dt:.3f} s "
      f"-> {trained / dt:.0f} frames/s (cache {cache}, bunch 1024)", flush=True)
