"""The oracle (oracle/tnet_oracle.c) pinned against golden vectors produced by the reference
CPU TNet (tests/golden/make_golden.py).  CPU-only."""
import os

import numpy as np
import pytest

import oracle as orc


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def _weights(g, prefix, nl):
    return [g[f"{prefix}W{k}"] for k in range(nl)], [g[f"{prefix}b{k}"] for k in range(nl)]


@pytest.mark.parametrize("name,keep_all", [("steps_tiny.npz", True), ("steps_slice.npz", False)])
def test_mlp_steps_cpu_semantics(golden_dir, name, keep_all):
    g = _load(golden_dir, name)
    dims = list(g["dims"])
    nl = len(dims) - 1
    B = int(g["bunch"])
    lr, wc = float(g["lr"]), float(g["wc"])
    W, b = _weights(g, "init_", nl)
    net = orc.MLP(W, b)
    X, lab = g["X"], g["labels"]
    nsteps = X.shape[0] // B
    for s in range(nsteps):
        Y, E = net.step(X[s * B:(s + 1) * B], lab[s * B:(s + 1) * B], lr, wc=wc, cpu_semantics=True)
        # outputs/errors: float tolerance vs MKL sgemm + float softmax of the reference
        np.testing.assert_allclose(Y, g[f"Y_{s}"], rtol=2e-4, atol=2e-6)
        np.testing.assert_allclose(E, g[f"E_{s}"], rtol=2e-4, atol=2e-6)
        if keep_all or s == nsteps - 1:
            Wr, br = _weights(g, f"step{s}_", nl)
            for k in range(nl):
                np.testing.assert_allclose(net.W[k], Wr[k], rtol=1e-4, atol=1e-6)
                np.testing.assert_allclose(net.b[k], br[k], rtol=1e-4, atol=1e-6)
    assert net.frames == int(g["frames"])
    np.testing.assert_allclose(net.xent, float(g["xent_sum"]), rtol=1e-6)


def test_gpu_semantics_reduce_to_cpu(golden_dir):
    """GRADDIVFRM=F, momentum 0 on the CuTNetLib update == CPU TNet THREADS=1 (run_test.GPU.sh:50)."""
    g = _load(golden_dir, "steps_tiny.npz")
    dims = list(g["dims"])
    nl = len(dims) - 1
    B = int(g["bunch"])
    W, b = _weights(g, "init_", nl)
    cpu, gpu = orc.MLP(W, b), orc.MLP(W, b)
    X, lab = g["X"], g["labels"]
    for s in range(X.shape[0] // B):
        sl = slice(s * B, (s + 1) * B)
        cpu.step(X[sl], lab[sl], 0.05, cpu_semantics=True)
        gpu.step(X[sl], lab[sl], 0.05, mmt=0.0, graddivfrm=False, cpu_semantics=False)
    for k in range(nl):
        np.testing.assert_allclose(gpu.W[k], cpu.W[k], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(gpu.b[k], cpu.b[k], rtol=1e-5, atol=1e-7)


def test_shuffle_permutations(golden_dir):
    g = _load(golden_dir, "shuffle.npz")
    for key in g.files:
        _, seed, n, cache, bunch = key.split("_")
        seed, n, cache, bunch = int(seed), int(n), int(cache), int(bunch)
        sched = orc.epoch_schedule([n], cache, bunch, seed).reshape(-1)
        # the reference harness adds one n-frame utterance into an n-capable cache: only the
        # first cache's bunches are emitted by it
        ref = g[key]
        np.testing.assert_array_equal(sched[: len(ref)], ref)


def test_epoch_schedule_counts(golden_dir):
    import json
    from tnet_amd import formats
    for name in ("epoch_mlp3.json", "epoch_mlp3_b256.json"):
        cfg = json.load(open(os.path.join(golden_dir, name)))
        rng = np.random.default_rng(cfg["corpus_seed"])
        lens = rng.integers(cfg["min_len"], cfg["max_len"] + 1, size=cfg["n_utts"])
        sched = orc.epoch_schedule(lens, cfg["cache"], cfg["bunch"], cfg["seed"])
        assert sched.size == cfg["frames"]
        assert len(np.unique(sched)) == sched.size


@pytest.mark.parametrize("name", ["epoch_mlp3.json", "epoch_mlp3_b256.json"])
def test_epoch_matches_reference_report(golden_dir, name):
    """Whole TNet epoch (cache fill/leftover/shuffle/bunching + SGD) vs the reference Report line."""
    import json
    from tnet_amd import formats
    cfg = json.load(open(os.path.join(golden_dir, name)))
    corpus = formats.synth_corpus(cfg["n_utts"], cfg["dim"], cfg["n_cls"], seed=cfg["corpus_seed"],
                                  min_len=cfg["min_len"], max_len=cfg["max_len"])
    layers = formats.round_trip_text(formats.gen_mlp_init(cfg["dims"], seed=cfg["init_seed"]), 6)
    X = np.concatenate(corpus.feats)
    L = np.concatenate(corpus.labels)
    sched = orc.epoch_schedule([len(l) for l in corpus.labels], cfg["cache"], cfg["bunch"], cfg["seed"])
    net = orc.MLP.from_layers(layers)
    for b in sched:
        net.step(X[b], L[b], cfg["lr"], cpu_semantics=True)
    assert net.frames == cfg["frames"]
    # the Report() line prints 6 significant digits
    np.testing.assert_allclose(net.xent, cfg["xent"], rtol=5e-6)
    np.testing.assert_allclose(100.0 * net.correct / net.frames, cfg["correct_pct"], atol=2e-5)


def test_epoch_schedule_leftover_filling_cache_is_an_error():
    # 500 rows, then 1100: 12 fill the cache, the 1088-row leftover is truncated to the whole
    # 512-row cache, leaving no space for the third utterance -> reference assert(cache_space > 0)
    with pytest.raises(ValueError):
        orc.epoch_schedule([500, 1100, 100], 512, 64, 1)
    assert orc.epoch_schedule([500, 1100], 512, 64, 1).shape == (8, 64)  # last leftover dropped
