#!/usr/bin/env python3
"""Is a training step host-bound?  Times the host's enqueue of K steps (Trainer.replay returns once every launch
is queued) against the same K steps' completion (after a synchronize): when enqueue ≈ completion the GPU waits on
the host.  Same network / cache / trainer set-up as bench.py.

usage: python tools/host_rate.py [--config mlp3] [--force-dp] [--steps 400]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import bench  # noqa: E402
import tnet_amd  # noqa: E402
from tnet_amd import Comm, Objective, Trainer  # noqa: E402
from tnet_amd._lib import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="mlp3")
    ap.add_argument("--force-dp", action="store_true")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--bunch", type=int, default=1024)
    a = ap.parse_args()
    dims = bench.CONFIGS[a.config]
    net = bench.build_network(dims)
    net.set_learn_rate(0.008)
    net.set_grad_div_frm(True)
    obj = Objective()
    cache = 65536
    tr = Trainer(net, obj, bunchsize=a.bunch, cachesize=cache, seed=123, randomize=True)
    comm = None
    if a.force_dp:
        comm = Comm(0, 1, Comm.unique_id())
        tr.set_comm(comm)
    X, L = bench.synth_frames(cache, dims[0], dims[-1], seed=1000)
    lib().tnet_trainer_prefill(tr.h, X.ctypes.data, X.shape[0], X.shape[1], X.shape[1], L.ctypes.data)
    tr.replay(100)
    tnet_amd.synchronize()
    out = {"config": a.config, "force_dp": a.force_dp, "steps": a.steps}
    for rep in range(3):
        t0 = time.perf_counter()
        tr.replay(a.steps)
        t1 = time.perf_counter()
        tnet_amd.synchronize()
        t2 = time.perf_counter()
        out[f"rep{rep}"] = {"host_enqueue_us_per_step": round(1e6 * (t1 - t0) / a.steps, 2),
                            "completion_us_per_step": round(1e6 * (t2 - t0) / a.steps, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
