#!/usr/bin/env python3
"""Frame accuracy of data-parallel training at 1, 2, 4 and 8 ranks (the
weak-scaling mode needs "matched frame accuracy" shown on a teacher-labelled set).

Every rank is a process on ONE GPU here (the 8-GPU node is the driver's), the gradients summed by
the host-transport communicator over gloo -- the same exchange protocol as the RCCL path
(GradExchange: per-layer sum, GRADDIVFRM over the global bunch, zero-gradient joins for uneven
shards), so the trajectory is the one an N-GPU run takes.  Network: BASELINE config 2's MLP3
(598:1024:135 sigmoid + softmax); data: a synthetic 598-dim N(0,1) corpus labelled by a fixed
random teacher MLP (learnable, tools/../formats.synth_corpus), utterances dealt round-robin to the
ranks (Platform.h:206-236), bunch 1024 frames PER RANK (global 1024 N), learning rate scaled
linearly with N (lr_N = N lr_1: the same step per epoch of frames; --scale sqrt: sqrt(N) lr_1).  After every epoch (one
TNetCu-style pass, fresh cache / shuffle seed per epoch, TNetCu.cc:330-441) rank 0 evaluates a
held-out set in cross-validation mode (TNetCu -c).

--newbob: the epochs are driven by the reference's newbob schedule (tools/train/
training_scheduler_xent.sh:56-214, restated in tnet_amd.newbob): after every epoch the held-out
cross-entropy decides accept (keep the weights) or reject (restore the previous best), halving starts
once an epoch improves the CV cross-entropy by less than START_HALVING_INC and training stops once a
halving epoch improves it by less than END_HALVING_INC (--end-halving-inc, the script's 0.1 by
default); --epochs is then MAX_ITER.  --warmup F: in the first epoch the learning rate ramps linearly
from lr_1 to lr_N over the first fraction F of the rank's utterances (the large-global-bunch runs
otherwise take their first steps at N times the single-GPU rate from random weights).

usage: python tools/dp_accuracy.py [--worlds 1,2,4,8] [--epochs 4] [--utts 800] [--lr 1.0]
       [--newbob] [--warmup 0.5] (worker mode is internal)"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import numpy as np  # noqa: E402

DIMS = [598, 1024, 135]
SEED = 7


def teacher(dim, n_cls, hidden=64):
    trng = np.random.default_rng(SEED + 1)
    return [trng.standard_normal((dim, hidden)).astype(np.float32) / np.sqrt(dim),
            trng.standard_normal((hidden, n_cls)).astype(np.float32) / np.sqrt(hidden) * 4.0]


def utterance(i, T, split):
    """utterance i of a split (0 train, 1 held-out), generated on its own seed (a rank makes only
    its shard)"""
    rng = np.random.default_rng(1000003 * (split + 1) + i)
    n = int(rng.integers(200, 1501))
    x = rng.standard_normal((n, DIMS[0])).astype(np.float32)
    h = np.tanh(x @ T[0]) @ T[1]
    return x, np.argmax(h, axis=1).astype(np.int32)


def worker(a):
    import torch
    import torch.distributed as dist

    import tnet_amd
    from tnet_amd import Network, Objective, Trainer, formats

    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    comm = None
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)

        def allreduce(v):
            dist.all_reduce(torch.from_numpy(v))

        comm = tnet_amd.Comm.host(rank, world, allreduce)
    transform = None
    if a.corpus == "ex01":
        # examples/01's own files (tests/golden/ex01): raw 23-dim FBANK through the native reader, the real
        # Hamm_dct_norm front end on the GPU (25/25 frame extension) -> 598 dims; the last 10 of the 100
        # utterances held out
        ex = os.path.join(REPO, "tests", "golden", "ex01")
        cwd = os.getcwd()
        os.chdir(ex)
        try:
            utts = [(x.copy(), lab.copy()) for _, x, lab, _, _ in
                    tnet_amd.FeatureReader("test.scp", mlf="test_3s.mlf", label_map="mono_state_phn_set_135_phn")]
        finally:
            os.chdir(cwd)
        transform = Network(path=os.path.join(ex, "Hamm_dct_norm"))
        mine = tnet_amd.shard_utterances(list(range(90)), rank, world)
        train = [utts[i] for i in mine]
        held = utts[90:] if rank == 0 else []
    else:
        T = teacher(DIMS[0], DIMS[-1])
        mine = tnet_amd.shard_utterances(list(range(a.utts)), rank, world)
        train = [utterance(i, T, 0) for i in mine]
        held = [utterance(i, T, 1) for i in range(a.cv_utts)] if rank == 0 else []
    from tnet_amd import newbob
    net = Network.from_layers(formats.gen_mlp_init(DIMS, seed=SEED + 101 * a.seed))
    lr = a.lr * {"linear": world, "sqrt": world ** 0.5, "none": 1.0}[a.scale]
    net.set_learn_rate(lr)
    net.set_grad_div_frm(True)
    nb = newbob.Newbob(repr(lr), a.bunch, max_iter=a.epochs, end_halving_inc=a.end_halving_inc,
                       start_halving_inc=a.start_halving_inc) if a.newbob else None
    best = None
    log = []
    t0 = time.time()

    def cv_eval():
        cobj = Objective()
        # the held-out set in bunches of --cv-bunch (default: the training bunch): a fixed value keeps the
        # evaluated frames the same for every world size (the cache drops the tail short of a bunch)
        cv = Trainer(net, cobj, bunchsize=a.cv_bunch or a.bunch, cachesize=a.cache, seed=0, randomize=False,
                     crossval=True)
        if transform is not None:
            cv.set_transform(transform, 25, 25)
        cv.train_corpus([x for x, _ in held], [y for _, y in held])
        return cobj.stats()

    def bcast_cv():
        """rank 0's held-out statistics, to every rank (the schedule's decisions must agree)"""
        v = np.zeros(3, np.float64)
        if rank == 0:
            v[:] = cv_eval()
        return comm.allreduce_host(v) if comm is not None else v

    if nb is not None:
        ce, cf, _ = bcast_cv()
        nb.initial("%.6g" % (ce / cf))
        best = [(W.copy(), b.copy()) for W, b in net.linear_params()]
    for ep in range(a.epochs):
        obj = Objective()
        tr = Trainer(net, obj, bunchsize=a.bunch, cachesize=a.cache, seed=1 + 1000 * ep + rank + 7919 * a.seed)
        if transform is not None:
            tr.set_transform(transform, 25, 25)
        if comm is not None:
            tr.set_comm(comm)
        ep_lr = float(nb.lrate) if nb is not None else lr
        if ep == 0 and a.warmup > 0 and world > 1:
            nw = max(1, int(a.warmup * len(train)))
            for k, (x, y) in enumerate(train):
                net.set_learn_rate(a.lr + (ep_lr - a.lr) * min(1.0, k / nw))
                tr.add_utterance(x, y)
            tr.finish()
        else:
            net.set_learn_rate(ep_lr)
            tr.train_corpus([x for x, _ in train], [y for _, y in train])
        err, frames, correct = obj.stats()
        st = np.array([err, frames, correct], np.float64)
        if comm is not None:
            st = comm.allreduce_host(st)
        rec = {"epoch": ep + 1, "lr": ep_lr, "train_xent_per_frame": st[0] / st[1],
               "train_acc": 100.0 * st[2] / st[1], "train_frames": int(st[1]), "steps_rank0": tr.steps}
        del tr
        ce, cf, cc = bcast_cv()
        rec.update(cv_xent_per_frame=ce / cf, cv_acc=100.0 * cc / cf, cv_frames=int(cf))
        if nb is not None:
            acc = nb.decide(ep + 1, "%.6g" % rec["train_xent_per_frame"], "%.6g" % (ce / cf), f"epoch{ep + 1}")
            rec["accepted"] = acc
            if acc:
                best = [(W.copy(), b.copy()) for W, b in net.linear_params()]
            else:                                   # the script reverts to the best network
                for k, (W, b) in enumerate(best):
                    net.set_params(2 * k, W, b)
        log.append(rec)
        if rank == 0 and a.progress:
            with open(a.progress, "a") as fh:
                fh.write(json.dumps(dict(rec, world=world, t=round(time.time() - t0, 1))) + "\n")
        if nb is not None and nb.done:
            break
    if nb is not None:
        for k, (W, b) in enumerate(best):
            net.set_params(2 * k, W, b)
        ce, cf, cc = bcast_cv()
        log.append({"final_best": True, "cv_xent_per_frame": ce / cf, "cv_acc": 100.0 * cc / cf})
    if rank == 0:
        print("RESULT " + json.dumps({"world": world, "corpus": a.corpus, "seed": a.seed, "lr": lr, "lr_scaling": a.scale,
                                      "newbob": a.newbob,
                                      "warmup": a.warmup, "end_halving_inc": a.end_halving_inc,
                                      "start_halving_inc": a.start_halving_inc,
                                      "bunch_per_rank": a.bunch,
                                      "global_bunch": a.bunch * world, "epochs": log,
                                      "wall_s": round(time.time() - t0, 1)}), flush=True)
    if comm is not None:
        dist.barrier()
        dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", nargs="?", default="launch", choices=["launch", "worker"])
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--utts", type=int, default=800)
    ap.add_argument("--cv-utts", type=int, default=40)
    ap.add_argument("--cv-bunch", type=int, default=0, help="held-out bunch size (0: --bunch)")
    ap.add_argument("--bunch", type=int, default=1024)
    ap.add_argument("--cache", type=int, default=16384)
    ap.add_argument("--lr", type=float, default=1.0)
    ap.add_argument("--scale", default="linear", choices=["linear", "sqrt", "none"],
                    help="lr_N = lr_1 N, lr_1 sqrt(N), or lr_1 (strong scaling: the global bunch stays the N=1 one)")
    ap.add_argument("--seed", type=int, default=0, help="run seed: the initial network and every cache shuffle")
    ap.add_argument("--newbob", action="store_true")
    ap.add_argument("--end-halving-inc", type=float, default=0.1)
    ap.add_argument("--start-halving-inc", type=float, default=0.5)
    ap.add_argument("--warmup", type=float, default=0.0)
    ap.add_argument("--progress", default="", help="rank 0 appends one JSON line per epoch to this file")
    ap.add_argument("--corpus", default="teacher", choices=["teacher", "ex01"],
                    help="teacher: the synthetic teacher-labelled corpus; ex01: examples/01's own files (90 train / "
                         "10 held-out utterances) through the real Hamm_dct_norm front end")
    a = ap.parse_args()
    if a.mode == "worker":
        worker(a)
        return
    out = []
    for world in [int(w) for w in a.worlds.split(",")]:
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(world),
                   OMP_NUM_THREADS="2")
        args = [sys.executable, os.path.abspath(__file__), "worker", "--epochs", str(a.epochs), "--utts",
                str(a.utts), "--cv-utts", str(a.cv_utts), "--bunch", str(a.bunch), "--cache", str(a.cache), "--lr",
                str(a.lr), "--scale", a.scale, "--end-halving-inc", str(a.end_halving_inc),
                "--start-halving-inc", str(a.start_halving_inc), "--warmup", str(a.warmup),
                "--progress", a.progress, "--corpus", a.corpus, "--seed", str(a.seed),
                "--cv-bunch", str(a.cv_bunch)]
        if a.newbob:
            args.append("--newbob")
        procs = [subprocess.Popen(args, env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                  text=True) for r in range(world)]
        res = None
        for r, p in enumerate(procs):
            o, e = p.communicate(timeout=1500)
            if p.returncode != 0:
                raise SystemExit(f"world {world} rank {r} failed:\n{e[-3000:]}")
            for line in o.splitlines():
                if line.startswith("RESULT "):
                    res = json.loads(line[7:])
        print(json.dumps(res), flush=True)
        out.append(res)
    print("SUMMARY " + json.dumps([{"world": r["world"], "lr": r["lr"], "cv_acc": [round(e["cv_acc"], 2) for e in r["epochs"]],
                                     "train_acc": [round(e["train_acc"], 2) for e in r["epochs"] if "train_acc" in e]}
                                    for r in out]), flush=True)


if __name__ == "__main__":
    main()
