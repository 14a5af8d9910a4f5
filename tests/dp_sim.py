"""Test helper: expected result of data-parallel training (the rounds protocol of
trainer.cpp DpPlanRound / CuTrainer::DrainCache) computed with the CPU oracle.

Rank r trains the utterance shard r::world with its own cache and shuffle seed.  Its k-th cache
drain is protocol round k: rounds k < d_r hold cachesize/bunch bunches (full caches), round d_r
holds the p_r bunches of the final partial drain, later rounds none.  Step j of a round trains
the concatenation (in rank order) of the j-th bunches of the ranks that still have one; the
update divides by the rows of that global bunch (GRADDIVFRM).
"""
from __future__ import annotations

import numpy as np


def rank_rounds(n_bunches: int, cachesize: int, bunch: int):
    """[(n, final)] protocol rounds of one rank that trains n_bunches over its epoch."""
    per = cachesize // bunch
    d, p = divmod(n_bunches, per)
    return [(per, False)] * d + [(p, True)]


def plan(rounds_per_rank):
    """Merge the ranks' rounds exactly as DpPlanRound does: list of rounds, each a list of
    steps, each the tuple of ranks training at that step."""
    world = len(rounds_per_rank)
    out, k = [], 0
    while True:
        row = [rounds_per_rank[r][k] if k < len(rounds_per_rank[r]) else (0, True) for r in range(world)]
        steps = max(n for n, _ in row)
        out.append([tuple(r for r in range(world) if row[r][0] > j) for j in range(steps)])
        if all(f for _, f in row):
            return out
        k += 1


def expected_dp_training(orc, layers, corpus, world, bunch, cachesize, seeds, lr, graddivfrm=True):
    """Oracle MLP after one data-parallel epoch; also returns per-rank bunch counts."""
    from tnet_amd import shard_utterances
    shards = [shard_utterances(range(len(corpus.feats)), r, world) for r in range(world)]
    X = [np.concatenate([corpus.feats[i] for i in sh]) for sh in shards]
    L = [np.concatenate([corpus.labels[i] for i in sh]) for sh in shards]
    sched = [orc.epoch_schedule([len(corpus.labels[i]) for i in sh], cachesize, bunch, seeds[r])
             for r, sh in enumerate(shards)]
    rounds = plan([rank_rounds(len(s), cachesize, bunch) for s in sched])
    net = orc.MLP.from_layers(layers)
    pos = [0] * world
    for rnd in rounds:
        for ranks in rnd:
            xs, ls = [], []
            for r in ranks:
                b = sched[r][pos[r]]
                pos[r] += 1
                xs.append(X[r][b])
                ls.append(L[r][b])
            net.step(np.concatenate(xs), np.concatenate(ls), lr, graddivfrm=graddivfrm)
    assert pos == [len(s) for s in sched]
    return net, [len(s) for s in sched], rounds
