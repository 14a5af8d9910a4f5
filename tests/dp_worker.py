"""Worker process of tests/test_gpu_dp.py: one data-parallel rank on the GPU, host-transport
communicator summing over torch.distributed/gloo.  Writes its final parameters to an npz.

usage: python dp_worker.py MODE OUT.npz   (RANK / WORLD_SIZE / MASTER_* in the environment)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
sys.path.insert(0, HERE)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import tnet_amd  # noqa: E402
from tnet_amd import DeviceArray, Network, Objective, Trainer, formats  # noqa: E402

import dp_cases  # noqa: E402


def main():
    mode, out = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce(a):
        dist.all_reduce(torch.from_numpy(a))

    comm = tnet_amd.Comm.host(rank, world, allreduce)
    res = {}
    if mode == "net":
        c = dp_cases.NET
        net = Network.from_layers(formats.gen_mlp_init(c["dims"], seed=c["init_seed"]))
        net.set_learn_rate(c["lr"])
        net.set_grad_div_frm(True)
        net.set_comm(comm)
        obj = Objective()
        for s, (X, L, active) in enumerate(dp_cases.net_bunches(world)):
            if rank in active:
                k = active.index(rank)
                B = c["bunch"]
                comm.set_step_rows(len(active) * B)
                net.train_bunch(obj, DeviceArray.from_numpy(X[k * B:(k + 1) * B]),
                                DeviceArray.vector(L[k * B:(k + 1) * B]))
                comm.set_step_rows(0)
            else:
                net.train_empty(comm, len(active) * c["bunch"])
        res["frames"] = obj.stats()[1]
    elif mode == "trainer":
        c = dp_cases.TRAINER
        corpus = dp_cases.trainer_corpus()
        net = Network.from_layers(formats.gen_mlp_init(c["dims"], seed=c["init_seed"]))
        net.set_learn_rate(c["lr"])
        net.set_grad_div_frm(c["gdf"])
        obj = Objective()
        tr = Trainer(net, obj, bunchsize=c["bunch"], cachesize=c["cache"], seed=c["seed"] + rank)
        tr.set_comm(comm)
        idx = tnet_amd.shard_utterances(range(len(corpus.feats)), rank, world)
        tr.train_corpus([corpus.feats[i] for i in idx], [corpus.labels[i] for i in idx])
        err, frames, correct = obj.stats()
        res.update(steps=tr.steps, empty_steps=tr.empty_steps, xent=err, frames=frames, correct=correct)
    elif mode == "full":
        c = dp_cases.FULL
        net = Network.from_layers(formats.gen_mlp_init(c["dims"], seed=c["init_seed"]))
        net.set_learn_rate(c["lr"])
        net.set_grad_div_frm(True)
        net.set_comm(comm)
        obj = Objective()
        b = c["bunch"] // world
        for X, L in dp_cases.full_bunches():
            net.train_bunch(obj, DeviceArray.from_numpy(X[rank * b:(rank + 1) * b]),
                            DeviceArray.vector(L[rank * b:(rank + 1) * b]))
        err, frames, correct = obj.stats()
        res.update(xent=err, frames=frames, correct=correct)
    else:
        raise SystemExit(f"unknown mode {mode}")
    arrs = {}
    for k, (W, b) in enumerate(net.linear_params()):
        arrs[f"W{k}"], arrs[f"b{k}"] = W, b
    np.savez(out, meta=np.array(json.dumps(res)), **arrs)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
