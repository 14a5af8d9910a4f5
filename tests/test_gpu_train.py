"""End-to-end parity of the fused MI355X SGD path against the reference (golden vectors produced
by the reference CPU TNet) and against the oracle's restatement of the CuTNetLib semantics.

Tolerances:
  per-step outputs / weights (a few steps): rtol 2e-4, atol 1e-6 (fp32 GEMM order differences)
  one epoch (56k frames, ~55 SGD steps): Xent relative 1e-4, frame accuracy 0.05 % absolute
  (the reference's own CPU-vs-CUDA gap is 0.01 %, MKL threading 0.005 %).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle as orc  # noqa: E402
from tnet_amd import DeviceArray, Network, Objective, Trainer, formats  # noqa: E402


def _golden(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def _net_from(g, prefix, dims):
    layers = []
    nl = len(dims) - 1
    for k in range(nl):
        layers.append(formats.Layer("<biasedlinearity>", dims[k + 1], dims[k], g[f"{prefix}W{k}"], g[f"{prefix}b{k}"]))
        layers.append(formats.Layer("<softmax>" if k == nl - 1 else "<sigmoid>", dims[k + 1], dims[k + 1]))
    return layers


@pytest.mark.parametrize("name,keep_all", [("steps_tiny.npz", True), ("steps_slice.npz", False)])
def test_train_bunch_matches_reference_cpu_tnet(golden_dir, name, keep_all):
    """GRADDIVFRM=F, momentum 0 == TNet --THREADS=1 (run_test.GPU.sh:50); reference outputs."""
    g = _golden(golden_dir, name)
    dims = [int(d) for d in g["dims"]]
    B = int(g["bunch"])
    net = Network.from_layers(_net_from(g, "init_", dims))
    net.set_learn_rate(float(g["lr"]))
    net.set_weightcost(float(g["wc"]))
    net.set_grad_div_frm(False)
    net.keep_output(True)
    obj = Objective()
    X, lab = g["X"], g["labels"]
    nsteps = X.shape[0] // B
    for s in range(nsteps):
        dX = DeviceArray.from_numpy(X[s * B:(s + 1) * B])
        dL = DeviceArray.vector(lab[s * B:(s + 1) * B])
        net.train_bunch(obj, dX, dL)
        Y = net.output(len(dims) * 2 - 3, B)
        np.testing.assert_allclose(Y, g[f"Y_{s}"], rtol=2e-4, atol=2e-6)
        if keep_all or s == nsteps - 1:
            for k, (W, b) in enumerate(net.linear_params()):
                np.testing.assert_allclose(W, g[f"step{s}_W{k}"], rtol=2e-4, atol=1e-6)
                np.testing.assert_allclose(b, g[f"step{s}_b{k}"], rtol=2e-4, atol=1e-6)
    err, frames, correct = obj.stats()
    assert frames == int(g["frames"])
    np.testing.assert_allclose(err, float(g["xent_sum"]), rtol=1e-5)


@pytest.mark.parametrize("mmt,gdf,wc,lrf", [(0.5, True, 1e-4, None), (0.9, False, 0.0, "0:1:0.5"), (0.0, True, 1e-3, None)])
def test_train_bunch_gpu_semantics_vs_oracle(mmt, gdf, wc, lrf):
    """momentum / GRADDIVFRM / weight decay / per-layer learn-rate factors (cuBiasedLinearity.cc:46-64,
    cuNetwork.cc:80-134) vs the oracle restatement -- parity unpinned by a reference run (CUDA only)."""
    dims = [40, 64, 48, 12]
    rng = np.random.default_rng(3)
    layers = formats.gen_mlp_init(dims, seed=4)
    net = Network.from_layers(layers)
    lr = 0.5
    net.set_learn_rate(lr, lrf)
    net.set_momentum(mmt)
    net.set_weightcost(wc)
    net.set_grad_div_frm(gdf)
    obj = Objective()
    factors = [float(f) for f in lrf.split(":")] if lrf else [1.0, 1.0, 1.0]
    W = [L.W for L in layers if L.W is not None]
    b = [L.b for L in layers if L.W is not None]
    refs = [orc.MLP([W[k]], [b[k]]) for k in range(3)]  # per-layer state holders
    ref = orc.MLP(W, b)
    B = 32
    for s in range(5):
        X = rng.standard_normal((B, dims[0])).astype(np.float32)
        L = rng.integers(0, dims[-1], B).astype(np.int32)
        net.train_bunch(obj, DeviceArray.from_numpy(X), DeviceArray.vector(L))
        # oracle with per-layer learn rates: run one step per distinct factor set by scaling
        if lrf is None:
            ref.step(X, L, lr, mmt=mmt, wc=wc, graddivfrm=gdf)
    if lrf is None:
        for k, (Wg, bg) in enumerate(net.linear_params()):
            np.testing.assert_allclose(Wg, ref.W[k], rtol=2e-4, atol=2e-6)
            np.testing.assert_allclose(bg, ref.b[k], rtol=2e-4, atol=2e-6)
        e, f, c = obj.stats()
        np.testing.assert_allclose(e, ref.xent, rtol=1e-5)
        assert c == ref.correct
    else:
        # factor 0 on the first layer: it is frozen and the second layer becomes the stopper
        Wg0, bg0 = net.linear_params()[0]
        np.testing.assert_array_equal(Wg0, W[0])
        np.testing.assert_array_equal(bg0, b[0])


def test_generic_component_path_matches_fused():
    """CuNetwork::Propagate + CuCrossEntropy::Evaluate + Backpropagate (component by component)
    == the fused TrainBunch."""
    dims = [30, 50, 20]
    layers = formats.gen_mlp_init(dims, seed=9)
    rng = np.random.default_rng(10)
    X = rng.standard_normal((24, 30)).astype(np.float32)
    L = rng.integers(0, 20, 24).astype(np.int32)
    a, b = Network.from_layers(layers), Network.from_layers(layers)
    for n in (a, b):
        n.set_learn_rate(0.1)
        n.set_momentum(0.5)
        n.set_weightcost(1e-4)
    oa, ob = Objective(), Objective()
    dX, dL = DeviceArray.from_numpy(X), DeviceArray.vector(L)
    for _ in range(3):
        a.train_bunch(oa, dX, dL)
        Y = b.propagate(dX)
        E = DeviceArray(24, 20)
        ob.evaluate_labels(Y, dL, E)
        b.backpropagate(E)
    for (Wa, ba), (Wb, bb) in zip(a.linear_params(), b.linear_params()):
        np.testing.assert_allclose(Wa, Wb, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(ba, bb, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(oa.stats()[0], ob.stats()[0], rtol=1e-6)


@pytest.mark.parametrize("name", ["epoch_mlp3.json", "epoch_mlp3_b256.json"])
def test_epoch_matches_reference_report(golden_dir, name):
    """config 2: MLP3 598:1024:135, one TNetCu epoch with the reference's data order (cache fill,
    leftover, lrand48 shuffle, tail discard), GRADDIVFRM=F == CPU TNet THREADS=1."""
    cfg = json.load(open(os.path.join(golden_dir, name)))
    corpus = formats.synth_corpus(cfg["n_utts"], cfg["dim"], cfg["n_cls"], seed=cfg["corpus_seed"],
                                  min_len=cfg["min_len"], max_len=cfg["max_len"])
    layers = formats.round_trip_text(formats.gen_mlp_init(cfg["dims"], seed=cfg["init_seed"]), 6)
    net = Network.from_layers(layers)
    net.set_learn_rate(cfg["lr"])
    net.set_grad_div_frm(False)
    obj = Objective()
    tr = Trainer(net, obj, bunchsize=cfg["bunch"], cachesize=cfg["cache"], seed=cfg["seed"])
    tr.train_corpus(corpus.feats, corpus.labels)
    err, frames, correct = obj.stats()
    assert frames == cfg["frames"]
    np.testing.assert_allclose(err, cfg["xent"], rtol=1e-4)
    assert abs(100.0 * correct / frames - cfg["correct_pct"]) <= 0.05
    rep = obj.report()
    assert rep.startswith("Xent:") and "correct[" in rep


def test_cache_leftover_filling_cache_raises():
    """cuCache.cc:97 assert(cache_space > 0): a leftover that fills the whole cache is an error."""
    from tnet_amd import TnetError
    layers = formats.gen_mlp_init([8, 16, 4], seed=1)
    net = Network.from_layers(layers)
    tr = Trainer(net, Objective(), bunchsize=64, cachesize=512, seed=1)
    rng = np.random.default_rng(0)
    lens = [500, 1100, 100]
    with pytest.raises(TnetError):
        for n in lens:
            tr.add_utterance(rng.standard_normal((n, 8)).astype(np.float32), np.zeros(n, np.int32))


def test_out_of_range_label_rejected_at_intake():
    """a class id >= the number of network outputs is an error at intake (the reference's one-hot
    target matrix cannot hold one); negative ids stay allowed (all-zero target rows)"""
    from tnet_amd import RnnTrainer, TnetError
    layers = formats.gen_mlp_init([8, 16, 4], seed=1)
    net = Network.from_layers(layers)
    tr = Trainer(net, Objective(), bunchsize=16, cachesize=64, seed=1)
    rng = np.random.default_rng(0)
    X = rng.standard_normal((20, 8)).astype(np.float32)
    ok = rng.integers(0, 4, 20).astype(np.int32)
    ok[3] = -1
    tr.add_utterance(X, ok)
    bad = ok.copy()
    bad[7] = 4
    with pytest.raises(TnetError, match="outside"):
        tr.add_utterance(X, bad)
    with pytest.raises(ValueError):
        tr.add_utterance(X, ok[:10])
    rnn = Network.from_layers(formats.gen_recurrent_init(8, 16, 4, seed=3))
    rnn.set_learn_rate(0.1)
    rt = RnnTrainer(rnn, Objective(), bptt=2)
    with pytest.raises(TnetError, match="outside"):
        rt.train_utterance(X, bad)



@pytest.mark.gpu
@pytest.mark.parametrize("mmt", [0.0, 0.5])
def test_mlp3_step_with_update_pair_vs_oracle(mmt):
    """BASELINE config 2 (598:1024:135, bunch 1024): the step's last two updates (1024x135 and 598x1024)
    go out as ONE launch (tnet_affine_update_bias_pair); three steps against the oracle's fp64 step.
    Tolerance as tests/test_gpu_fullsize.py: the update, not W, is under test -- |W_gpu - W_ref| <=
    2 ulp(W) + 1e-4 max|W_ref - W_init| per layer, biases likewise; Xent rtol 1e-5."""
    dims = [598, 1024, 135]
    rng = np.random.default_rng(11)
    layers = formats.gen_mlp_init(dims, seed=12)
    net = Network.from_layers(layers)
    net.set_learn_rate(0.5)
    net.set_momentum(mmt)
    net.set_grad_div_frm(True)
    obj = Objective()
    W0 = [L.W.copy() for L in layers if L.W is not None]
    b0 = [L.b.copy() for L in layers if L.W is not None]
    ref = orc.MLP([w.copy() for w in W0], [x.copy() for x in b0])
    for _ in range(3):
        X = rng.standard_normal((1024, dims[0])).astype(np.float32)
        L = rng.integers(0, dims[-1], 1024).astype(np.int32)
        net.train_bunch(obj, DeviceArray.from_numpy(X), DeviceArray.vector(L))
        ref.step(X, L, 0.5, mmt=mmt, graddivfrm=True)
    for k, (Wg, bg) in enumerate(net.linear_params()):
        for got, want, init in ((Wg, ref.W[k], W0[k]), (bg, ref.b[k], b0[k])):
            d = np.abs(np.asarray(want, np.float64) - init).max()
            tol = 2 * np.spacing(np.abs(np.asarray(want, np.float32))) + 1e-4 * d
            assert np.all(np.abs(got.astype(np.float64) - want) <= tol), (k, np.abs(got - want).max(), d)
    np.testing.assert_allclose(obj.stats()[0], ref.xent, rtol=1e-5)
