"""Shared data-parallel test cases (tests/test_gpu_dp.py and its worker processes)."""
import numpy as np

from tnet_amd import formats

# network level, GRADDIVFRM=T: step 2 is trained by rank 0 alone (rank 1 joins with a zero gradient)
NET = dict(dims=[40, 96, 96, 12], init_seed=5, lr=0.5, bunch=64, steps=4, solo_step=2)

# trainer level, uneven shards: 9 utterances round-robin -> rank 0 gets 5, rank 1 gets 4 (and fewer
# frames), so rank 1 reaches its final drain first and joins the remaining steps empty
TRAINER = dict(dims=[40, 96, 96, 12], init_seed=7, lr=0.004, gdf=False, bunch=64, cache=512, seed=123,
               n_utts=9, corpus_seed=3, min_len=100, max_len=450)


def net_bunches(world):
    """[(X [len(active)*B x d], labels, active ranks)] per step."""
    rng = np.random.default_rng(11)
    out = []
    for s in range(NET["steps"]):
        active = [0] if s == NET["solo_step"] else list(range(world))
        n = len(active) * NET["bunch"]
        X = rng.standard_normal((n, NET["dims"][0])).astype(np.float32)
        L = rng.integers(0, NET["dims"][-1], n).astype(np.int32)
        out.append((X, L, active))
    return out


def trainer_corpus():
    c = TRAINER
    return formats.synth_corpus(c["n_utts"], c["dims"][0], c["dims"][-1], seed=c["corpus_seed"],
                                min_len=c["min_len"], max_len=c["max_len"])


# BASELINE config 3 at full network size through the data-parallel protocol: 440 -> 2048x5 -> 4000, the
# global bunch of 1024 frames split over 8 ranks (128 each: the reference's Platform semantics,
# Platform.h:159-160, bunch / N per worker), GRADDIVFRM=T over the global bunch, two steps
FULL = dict(dims=[440, 2048, 2048, 2048, 2048, 2048, 4000], init_seed=3, lr=1.0, bunch=1024, steps=2, world=8)


def full_bunches():
    """[(X [1024 x 440], labels)] per step -- the global bunches"""
    rng = np.random.default_rng(17)
    B, d, n = FULL["bunch"], FULL["dims"][0], FULL["dims"][-1]
    return [(rng.standard_normal((B, d)).astype(np.float32), rng.integers(0, n, B).astype(np.int32))
            for _ in range(FULL["steps"])]
