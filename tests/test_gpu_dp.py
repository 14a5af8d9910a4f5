"""Data-parallel path on the GPU: two ranks (processes) on one device, weight gradients summed by
the host-transport communicator over gloo (the RCCL communicator needs one GPU per rank; its
world-1 case is covered below).  Expected results come from the CPU oracle on the global bunches
(tests/dp_sim.py).  Tolerance: rtol 2e-4 / atol 1e-6 on parameters (fp32 GEMM order + the two
partial gradient sums vs one)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dp_cases  # noqa: E402
import dp_sim  # noqa: E402
import oracle as orc  # noqa: E402
from tnet_amd import Comm, DeviceArray, Network, Objective, Trainer, formats  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(mode, tmp_path, world=2, shard="0", inline="0"):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               OMP_NUM_THREADS="1", TNET_DP_SHARD=shard, TNET_DP_HOST_INLINE=inline)
    outs = [str(tmp_path / f"{mode}_r{r}.npz") for r in range(world)]
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), mode, outs[r]],
                              env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(world)]
    for p in procs:
        try:
            _, e = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-4000:]
    res = []
    for o in outs:
        z = np.load(o, allow_pickle=False)
        res.append((json.loads(str(z["meta"])), {k: z[k] for k in z.files if k != "meta"}))
    return res


def _assert_params(got, net, rtol=2e-4, atol=1e-6):
    for k in range(len(net.W)):
        np.testing.assert_allclose(got[f"W{k}"], net.W[k], rtol=rtol, atol=atol)
        np.testing.assert_allclose(got[f"b{k}"], net.b[k], rtol=rtol, atol=atol)


@pytest.mark.parametrize("world,shard,inline", [(2, "0", "0"), (2, "1", "0"), (3, "1", "0"), (3, "1", "1")])
def test_dp_network_ranks_match_global_bunch(tmp_path, world, shard, inline):
    """shard "1": the sharded apply (reduce, each rank updates its shard + the tails, the parameter
    blocks gathered back) -- RcclExchange's protocol, emulated over the host transport; world 3
    leaves tails (blocks whose size is not a multiple of 4 x 3 elements)"""
    c = dp_cases.NET
    ranks = _run_ranks("net", tmp_path, world, shard, inline)
    # every rank holds identical parameters
    for r in range(1, world):
        for k in ranks[0][1]:
            np.testing.assert_array_equal(ranks[0][1][k], ranks[r][1][k])
    net = orc.MLP.from_layers(formats.gen_mlp_init(c["dims"], seed=c["init_seed"]))
    for X, L, _ in dp_cases.net_bunches(world):
        net.step(X, L, c["lr"], graddivfrm=True)
    _assert_params(ranks[0][1], net)
    assert ranks[0][0]["frames"] == c["bunch"] * c["steps"]
    for r in range(1, world):
        assert ranks[r][0]["frames"] == c["bunch"] * (c["steps"] - 1)


@pytest.mark.parametrize("shard,inline", [("0", "0"), ("1", "0"), ("1", "1")])
def test_dp_trainer_uneven_shards(tmp_path, shard, inline):
    """inline "1": every layer's reduction, apply and parameter gather in turn (RcclExchange's order),
    with one rank training bunches while the other joins with zero gradients (TrainEmpty): the two
    must issue the same collective sequence or the host all-reduces pair up wrongly"""
    c = dp_cases.TRAINER
    ranks = _run_ranks("trainer", tmp_path, 2, shard, inline)
    for k in ranks[0][1]:
        np.testing.assert_array_equal(ranks[0][1][k], ranks[1][1][k])
    corpus = dp_cases.trainer_corpus()
    layers = formats.gen_mlp_init(c["dims"], seed=c["init_seed"])
    net, nb, rounds = dp_sim.expected_dp_training(orc, layers, corpus, 2, c["bunch"], c["cache"],
                                                  [c["seed"], c["seed"] + 1], c["lr"], graddivfrm=c["gdf"])
    assert nb[0] > nb[1], "the case must exercise unequal shards"
    total_steps = sum(len(r) for r in rounds)
    for r in range(2):
        assert ranks[r][0]["steps"] == nb[r]
        assert ranks[r][0]["steps"] + ranks[r][0]["empty_steps"] == total_steps
    _assert_params(ranks[0][1], net)
    np.testing.assert_allclose(ranks[0][0]["xent"] + ranks[1][0]["xent"], net.xent, rtol=1e-4)
    assert ranks[0][0]["frames"] + ranks[1][0]["frames"] == net.frames


@pytest.mark.parametrize("shard", ["0", "1"])
def test_dp_rccl_world1_equals_local_update(monkeypatch, shard):
    """RCCL communicator at world 1: the split ComputeGradient -> all-reduce -> ApplyGradient path
    gives the fused local update's result (shard "1": the reduce-scatter -> shard apply -> in-place
    all-gather form, one rank)."""
    c = dp_cases.NET
    monkeypatch.setenv("TNET_DP_SHARD", shard)
    comm = Comm(0, 1, Comm.unique_id())
    nets = []
    for use_comm in (False, True):
        net = Network.from_layers(formats.gen_mlp_init(c["dims"], seed=c["init_seed"]))
        net.set_learn_rate(c["lr"])
        net.set_momentum(0.5)
        if use_comm:
            net.set_comm(comm)
        obj = Objective()
        for X, L, active in dp_cases.net_bunches(1):
            net.train_bunch(obj, DeviceArray.from_numpy(X), DeviceArray.vector(L))
        nets.append(net.linear_params())
    for (W0, b0), (W1, b1) in zip(*nets):
        np.testing.assert_allclose(W1, W0, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(b1, b0, rtol=1e-5, atol=1e-7)
    v = comm.allreduce_host(np.array([1.5, -2.0]))
    assert v.tolist() == [1.5, -2.0]


def _assert_update_close(after_gpu, after_ref, before, rtol, what):
    ref = np.asarray(after_ref, np.float32)
    upd = np.abs(ref.astype(np.float64) - before)
    tol = 2.0 * np.spacing(np.abs(ref)).astype(np.float64) + rtol * upd.max()
    worst = float((np.abs(np.asarray(after_gpu, np.float64) - ref) / tol).max())
    assert worst <= 1.0, (what, worst)


def test_dp_rccl_reserved_cus_full_size(monkeypatch):
    """The RCCL exchange's CU reservation (TNET_DP_RESERVE_CUS, explicit at world 1): from the first
    reduction of a step to WaitAll the 2048^2 GEMMs run stream-K over CUs - 8 workgroups (split tiles
    combined in-launch).  Two full-size steps through the communicator match the oracle's steps with the
    tolerance of tests/test_gpu_fullsize.py (2 ulp + 1e-4 of the largest update), and differ from the
    unreserved local run in summation order only (evidence the stream-K path ran)."""
    dims, B, lr = [440, 2048, 2048, 2048, 135], 1024, 1.0
    layers = formats.gen_mlp_init(dims, seed=3)
    monkeypatch.setenv("TNET_DP_RESERVE_CUS", "8")
    comm = Comm(0, 1, Comm.unique_id())
    rng = np.random.default_rng(11)
    bunches = [(rng.standard_normal((B, dims[0])).astype(np.float32), rng.integers(0, dims[-1], B).astype(np.int32))
               for _ in range(2)]
    runs = []
    for use_comm in (False, True):
        net = Network.from_layers(layers)
        net.set_learn_rate(lr)
        net.set_grad_div_frm(True)
        if use_comm:
            net.set_comm(comm)
        obj = Objective()
        for X, L in bunches:
            net.train_bunch(obj, DeviceArray.from_numpy(X), DeviceArray.vector(L))
        runs.append((net.linear_params(), obj.stats()))
    ref = orc.MLP.from_layers(layers)
    W0 = [w.astype(np.float64) for w in ref.W]
    b0 = [b.astype(np.float64) for b in ref.b]
    for X, L in bunches:
        ref.step(X, L, lr)
    for params, stats in runs:
        for k, (W, b) in enumerate(params):
            _assert_update_close(W, ref.W[k], W0[k], 1e-4, f"layer {k} W")
            _assert_update_close(b, ref.b[k], b0[k], 1e-4, f"layer {k} b")
        np.testing.assert_allclose(stats[0], ref.xent, rtol=1e-5)
    assert any(not np.array_equal(runs[0][0][k][0], runs[1][0][k][0]) for k in (1, 2))


@pytest.mark.parametrize("shard", ["0", "1"])
def test_dp_config3_full_size_eight_ranks(tmp_path, shard):
    """BASELINE config 3's network at FULL size through the data-parallel exchange: 440 -> 2048x5 -> 4000,
    8 ranks (processes on one GPU, host transport over gloo -- RCCL needs a GPU per rank), 128 frames
    each of a global bunch of 1024 (Platform.h:159-160: bunch / N per worker), GRADDIVFRM=T over the
    global bunch, two steps; shard "1": reduce-scatter + sharded apply + all-gather (TNET_DP_SHARD=1).
    Every rank must hold bit-identical parameters, equal to the oracle's two steps on the global bunches
    within tests/test_gpu_fullsize.py's bound (2 ulp(W) + 1e-4 of the largest update per layer); the
    ranks' summed cross-entropy within 1e-5 of the oracle's."""
    c = dp_cases.FULL
    world = c["world"]
    ranks = _run_ranks("full", tmp_path, world, shard)
    for r in range(1, world):
        for k in ranks[0][1]:
            np.testing.assert_array_equal(ranks[0][1][k], ranks[r][1][k], err_msg=f"rank {r} {k}")
    layers = formats.gen_mlp_init(c["dims"], seed=c["init_seed"])
    ref = orc.MLP.from_layers(layers)
    W0 = [w.astype(np.float64) for w in ref.W]
    b0 = [b.astype(np.float64) for b in ref.b]
    for X, L in dp_cases.full_bunches():
        ref.step(X, L, c["lr"], graddivfrm=True)
    for k in range(len(ref.W)):
        _assert_update_close(ranks[0][1][f"W{k}"], ref.W[k], W0[k], 1e-4, f"layer {k} W")
        _assert_update_close(ranks[0][1][f"b{k}"], ref.b[k], b0[k], 1e-4, f"layer {k} b")
    assert sum(r[0]["frames"] for r in ranks) == c["bunch"] * c["steps"]
    np.testing.assert_allclose(sum(r[0]["xent"] for r in ranks), ref.xent, rtol=1e-5)
