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


# ---------------------------------------------------------------------------------------------
# feature front end: the numpy restatement vs the reference CPU TFeaCat (tests/golden/make_frontend.py)
# ---------------------------------------------------------------------------------------------

def _frontend_inputs():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "make_frontend", os.path.join(os.path.dirname(__file__), "golden", "make_frontend.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    from tnet_amd import formats
    corpus = formats.synth_corpus(**mf.CORPUS)
    layers = formats.round_trip_text(formats.gen_frontend_transform(**mf.TRANSFORM), 9)
    return mf, corpus, layers


def test_frontend_oracle_vs_reference_tfeacat(golden_dir):
    """Hamm_dct_norm-structured transform, frame extension 25/25: full output of two utterances
    (abs 1e-5; values up to ~10) and float64 sum / sum of squares of all 40 (rel 1e-6)."""
    mf, corpus, layers = _frontend_inputs()
    g = _load(golden_dir, "frontend_feacat.npz")
    for k, x in enumerate(corpus.feats):
        y = orc.frontend_forward(layers, x, 25, 25)
        assert y.shape == (int(g["rows"][k]), 598)
        if k in mf.FULL:
            np.testing.assert_allclose(y, g[f"Y_{k}"], rtol=0, atol=1e-5)
        y = y.astype(np.float64)
        assert abs(y.sum() - g["sum"][k]) <= 1e-6 * np.abs(y).sum()
        assert abs((y ** 2).sum() - g["sumsq"][k]) <= 1e-6 * g["sumsq"][k]


def test_frontend_decode_oracle_vs_reference_tfeacat(golden_dir):
    """decode.sh's TFeaCat call (transform + MLP + GMMBYPASS sqrt(-2 ln p), TFeaCat.cc:236-243)."""
    from tnet_amd import formats
    mf, corpus, layers = _frontend_inputs()
    g = _load(golden_dir, "frontend_decode.npz")
    mlp = formats.round_trip_text(formats.gen_mlp_init(mf.EPOCH["dims"], seed=mf.EPOCH["init_seed"]), 6)
    net = orc.MLP.from_layers(mlp)
    for k in (mf.DECODE, 0, 5):
        p = net.forward(orc.frontend_forward(layers, corpus.feats[k], 25, 25)).astype(np.float64)
        y = np.sqrt(-2.0 * np.log(p))
        if k == mf.DECODE:
            np.testing.assert_allclose(y, g[f"Y_{k}"], rtol=1e-4, atol=1e-5)
        assert abs(y.sum() - g["sum"][k]) <= 1e-5 * np.abs(y).sum()


def test_frontend_component_restatement_edges():
    """<copy> (1-based in the file, out-of-range -> +inf as _rearrange), <expand> clamping with
    asymmetric offsets, <log>, and the .nnet text round trip of every front-end tag."""
    from tnet_amd import formats
    rng = np.random.default_rng(3)
    x = rng.random((7, 5)).astype(np.float32) + 0.1
    cp = formats.Layer("<copy>", 4, 5, extra={"indices": np.array([4, 0, 0, 9])})
    y = orc.frontend_component(cp, x)
    np.testing.assert_array_equal(y[:, :3], x[:, [4, 0, 0]])
    assert np.isinf(y[:, 3]).all()
    ex = formats.Layer("<expand>", 15, 5, extra={"offsets": np.array([-3, 0, 2])})
    y = orc.frontend_component(ex, x)
    np.testing.assert_array_equal(y[0, :5], x[0])
    np.testing.assert_array_equal(y[1, :5], x[0])
    np.testing.assert_array_equal(y[6, 10:], x[6])
    np.testing.assert_array_equal(y[4, 10:], x[6])
    np.testing.assert_allclose(orc.frontend_component(formats.Layer("<log>", 5, 5), x), np.log(x), rtol=1e-6)
    layers = formats.gen_frontend_transform(dim=5, context=2, n_dct=3, seed=1) + [cp, formats.Layer("<log>", 4, 4)]
    back = formats.round_trip_text(layers, 9)
    assert [L.tag for L in back] == [L.tag for L in layers]
    np.testing.assert_array_equal(back[-2].extra["indices"], cp.extra["indices"])
    np.testing.assert_allclose(back[3].W, layers[3].W, rtol=1e-7)
