"""Data-parallel host logic on CPU, world_size 2 over gloo (no GPU).

Runs the PRODUCT's step planner (trainer.cpp DpPlanRound through tnet_dp_plan_round) in two
processes whose host-transport communicator sums over torch.distributed/gloo, and checks it
against the pure-Python statement of the protocol in tests/dp_sim.py, plus utterance sharding.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dp_sim  # noqa: E402

# per rank: the (n, final) rounds it submits; rank 1 runs out of utterances two drains early
SCENARIO = {0: [(4, False), (4, False), (4, False), (2, True)],
            1: [(4, False), (3, True), (0, True), (0, True)]}

WORKER = r'''
import os, sys, json
import numpy as np
import torch, torch.distributed as dist
sys.path.insert(0, os.path.join(sys.argv[1], "nnet-asr_amd"))
import tnet_amd
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
def allreduce(a):
    t = torch.from_numpy(a)
    dist.all_reduce(t)
comm = tnet_amd.Comm.host(rank, world, allreduce)
rounds = json.loads(sys.argv[2])[str(rank)]
out = []
for n, final in rounds:
    steps, allf = comm.plan_round(n, final)
    out.append([steps.tolist(), allf])
    if allf:
        break
# device-free float32 + float64 sums through the same callback
v = comm.allreduce_host(np.array([rank + 1.0, 2.0]))
print(json.dumps({"rounds": out, "sum": v.tolist()}))
dist.destroy_process_group()
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_utterances_round_robin():
    from tnet_amd import shard_utterances
    assert shard_utterances(range(7), 0, 3) == [0, 3, 6]
    assert shard_utterances(range(7), 2, 3) == [2, 5]
    allr = sorted(sum((shard_utterances(range(11), r, 4) for r in range(4)), []))
    assert allr == list(range(11))
    with pytest.raises(ValueError):
        shard_utterances(range(3), 2, 2)


def test_rank_rounds_and_plan():
    assert dp_sim.rank_rounds(10, 1024, 256) == [(4, False), (4, False), (2, True)]
    assert dp_sim.rank_rounds(8, 1024, 256) == [(4, False), (4, False), (0, True)]
    p = dp_sim.plan([[(4, False), (2, True)], [(3, True)]])
    assert p == [[(0, 1), (0, 1), (0, 1), (0,)], [(0,), (0,)]]


def test_dp_plan_gloo_world2():
    import json
    port = _free_port()
    env_base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2",
                    OMP_NUM_THREADS="1")
    repo = os.path.dirname(HERE)
    procs = [subprocess.Popen([sys.executable, "-c", WORKER, repo, json.dumps(SCENARIO)],
                              env=dict(env_base, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for r in range(2)]
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e[-3000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    expected = dp_sim.plan([SCENARIO[0], SCENARIO[1]])
    for o in outs:
        got = [[c for c in steps] for steps, _ in o["rounds"]]
        assert got == [[len(s) for s in rnd] for rnd in expected]
        assert [f for _, f in o["rounds"]] == [False] * (len(expected) - 1) + [True]
        assert o["sum"] == [3.0, 4.0]


@pytest.mark.parametrize("n", [0, 1, 3, 4, 7, 12, 23, 96, 135, 440 * 2048, 2048 * 4000 + 5])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_ranges_cover_every_element_once(n, world):
    """the sharded apply's split (trainer/gradexchange ShardRanges through tnet_dp_shard_ranges):
    the ranks' shards are disjoint, 16-byte aligned and equal; the tail (applied by every rank) and
    the shards together cover [0, n) exactly once per element"""
    import ctypes as C
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "nnet-asr_amd"))
    from tnet_amd._lib import check, lib
    owner = np.zeros(n, np.int32)
    tails = []
    for r in range(world):
        lo, hi, cnt = (C.c_long * 2)(), (C.c_long * 2)(), C.c_int()
        check(lib().tnet_dp_shard_ranges(n, r, world, lo, hi, C.byref(cnt)))
        rng = [(lo[k], hi[k]) for k in range(cnt.value)]
        for a, b in rng:
            assert 0 <= a <= b <= n
        c = (n // (4 * world)) * 4
        if c > 0:
            assert rng[0] == (r * c, r * c + c) and (r * c) % 4 == 0
            owner[r * c:r * c + c] += 1
        tail = [t for t in rng if t[0] >= c * world]
        tails.append(tail)
    main = (n // (4 * world)) * 4 * world
    assert all(t == tails[0] for t in tails)
    assert tails[0] == ([(main, n)] if main < n else [])
    owner[main:] += 1
    assert np.all(owner == 1)


CHECK_WORKER = r'''
import os, sys, json
import numpy as np
import torch, torch.distributed as dist
sys.path.insert(0, os.path.join(sys.argv[1], "nnet-asr_amd"))
from tnet_amd import dpcheck
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
def allreduce64(a):
    dist.all_reduce(torch.from_numpy(a))
def gather(res):
    got = [None] * world
    dist.all_gather_object(got, res)
    return got
sizes = [2048 * 7 + 3, 135, 1]
local = [np.random.default_rng(100 * r + i).standard_normal(n).astype(np.float32)
         for i, n in enumerate(sizes) for r in [rank]]
every = [[np.random.default_rng(100 * r + i).standard_normal(n).astype(np.float32) for r in range(world)]
         for i, n in enumerate(sizes)]
true_sum = [np.sum(np.stack(e), 0, dtype=np.float32) for e in every]
out = {}
# all-reduce form: every element reduced
out["allreduce"] = dpcheck.merge_ranks(gather(dpcheck.compare_reduction(list(zip(local, true_sum)), allreduce64)))
# sharded form: only this rank's shard + the tail reduced (NaN elsewhere), the ShardRanges split
def sharded(s, n):
    c = (n // (4 * world)) * 4
    r = np.full(n, np.nan, np.float32)
    r[rank * c:rank * c + c] = s[rank * c:rank * c + c]
    r[c * world:] = s[c * world:]
    return r
out["shard"] = dpcheck.merge_ranks(gather(dpcheck.compare_reduction(
    [(l, sharded(s, len(s))) for l, s in zip(local, true_sum)], allreduce64)))
# a stale operand: rank 1's reduction of block 0 missed its own contribution (what fence-free events could cause)
bad = [s.copy() for s in true_sum]
if rank == 1:
    bad[0] = bad[0] - local[0]
out["stale"] = dpcheck.merge_ranks(gather(dpcheck.compare_reduction(list(zip(local, bad)), allreduce64)))
print(json.dumps(out))
dist.destroy_process_group()
'''


def test_reduction_check_gloo_world2():
    """bench.py's rccl_check logic (tnet_amd/dpcheck.py) over gloo at world 2: the reduced gradients of both exchange
    forms (all-reduce; reduce-scatter with the rank's shard + tail) pass against the float64 sum of the local blocks,
    and a reduction that lost one rank's contribution on one rank is caught (ok False, the worst block named)"""
    import json
    port = _free_port()
    env_base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2", OMP_NUM_THREADS="1")
    repo = os.path.dirname(HERE)
    procs = [subprocess.Popen([sys.executable, "-c", CHECK_WORKER, repo], env=dict(env_base, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e[-3000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    for o in outs:
        assert o["allreduce"]["ok"] and o["allreduce"]["max_rel_err"] < 1e-6 and o["allreduce"]["blocks"] == 3
        assert o["shard"]["ok"] and o["shard"]["max_rel_err"] < 1e-6
        n0 = 2048 * 7 + 3
        c = (n0 // 8) * 4
        c1 = (135 // 8) * 4
        assert o["shard"]["elements_per_rank"][0] == (c + n0 - 2 * c) + (c1 + 135 - 2 * c1) + 1
        assert not o["stale"]["ok"] and o["stale"]["worst_block"] == 0 and o["stale"]["max_rel_err"] > 0.1
