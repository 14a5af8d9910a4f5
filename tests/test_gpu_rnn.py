"""Recurrent path (BASELINE config 5: Elman RNN trained frame by frame with truncated BPTT, the
TRecurrentCu loop) on the GPU vs the oracle's restatement of CuRecurrent / TRecurrentCu.

CuRecurrent is CUDA-only in the reference (no CPU counterpart), so parity is against the
restatement (oracle/tnet_oracle.c orc_rnn_utterance) -- "parity restated", not reference-run.
Tolerances: single-frame kernels rtol 1e-5; after whole utterances (hundreds of sequential
per-frame SGD updates, each amplifying fp32 rounding differences) parameters rtol 2e-3 /
atol 2e-5 and summed cross-entropy rtol 1e-4.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle as orc  # noqa: E402
from tnet_amd import DeviceArray, Network, Objective, RnnTrainer, formats, synchronize  # noqa: E402
from tnet_amd._lib import check, lib  # noqa: E402


def S():
    return lib().tnet_stream()


@pytest.mark.parametrize("K,N,act", [(1, 1, 0), (952, 512, 1), (440, 135, 0), (2100, 70, 1)])
def test_gemv_rowvec(K, N, act):
    rng = np.random.default_rng(K + N)
    v = rng.standard_normal(K).astype(np.float32)
    W = (0.05 * rng.standard_normal((K, N))).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    dv, dW, db = DeviceArray.from_numpy(v.reshape(1, -1)), DeviceArray.from_numpy(W), DeviceArray.vector(b)
    y = DeviceArray(1, N)
    ws = DeviceArray(1, max(1, lib().tnet_gemv_workspace(K, N) // 4))
    check(lib().tnet_gemv_rowvec(dv.ptr, K, dW.ptr, dW.stride, db.ptr, y.ptr, N, act, ws.ptr, S()))
    a = b + v.astype(np.float64) @ W
    np.testing.assert_allclose(y.numpy().reshape(-1), a if act == 0 else 1 / (1 + np.exp(-a)), rtol=1e-5,
                               atol=1e-5)


@pytest.mark.parametrize("r0,nrows,n,beta,sig", [(0, 440, 512, 0.0, False), (440, 512, 512, 1.0, True),
                                                  (3, 7, 13, 0.5, True)])
def test_gemv_rows(r0, nrows, n, beta, sig):
    rng = np.random.default_rng(nrows)
    W = rng.standard_normal((r0 + nrows, n)).astype(np.float32)
    x = rng.standard_normal(n).astype(np.float32)
    y0 = rng.standard_normal(nrows).astype(np.float32)
    s = rng.random(nrows).astype(np.float32)
    dW, dx, dy, ds = (DeviceArray.from_numpy(a.reshape(1, -1) if a.ndim == 1 else a) for a in (W, x, y0, s))
    check(lib().tnet_gemv_rows(dW.ptr, dW.stride, r0, nrows, n, dx.ptr, dy.ptr, beta, ds.ptr if sig else None, S()))
    ref = beta * y0 + W[r0:].astype(np.float64) @ x
    if sig:
        ref = ref * s * (1 - s)
    np.testing.assert_allclose(dy.numpy().reshape(-1), ref, rtol=1e-5, atol=1e-5)


def test_recurrent_text_round_trip(tmp_path):
    layers = formats.gen_recurrent_init(20, 16, 9, seed=3)
    net = Network.from_layers(layers)
    assert net.components()[0] == ("<recurrent>", 20, 16)
    W, b = net.recurrent_params(0)
    np.testing.assert_array_equal(W, layers[0].W)
    p = str(tmp_path / "rnn.nnet")
    net.write(p)
    back = formats.read_nnet(p)
    assert back[0].tag == "<recurrent>" and back[0].W.shape == (36, 16)
    np.testing.assert_allclose(back[0].W, layers[0].W, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("bptt,mmt,wc", [(4, 0.0, 0.0), (2, 0.5, 1e-4), (0, 0.0, 0.0)])
def test_rnn_trainer_matches_oracle(bptt, mmt, wc):
    """Two utterances through TRecurrentCu semantics (history reset per utterance), the per-frame launch chain."""
    nIn, H, Sd, lr = 24, 32, 10, 0.05
    rng = np.random.default_rng(bptt)
    layers = formats.round_trip_text(formats.gen_recurrent_init(nIn, H, Sd, seed=7), 9)
    feats = [rng.standard_normal((T, nIn)).astype(np.float32) for T in (60, 45)]
    labels = [rng.integers(0, Sd, len(f)).astype(np.int32) for f in feats]
    net = Network.from_layers(layers)
    net.set_learn_rate(lr)
    net.set_momentum(mmt)
    net.set_weightcost(wc)
    obj = Objective()
    tr = RnnTrainer(net, obj, bptt=bptt)
    tr.train_corpus(feats, labels)
    m = orc.RNN(layers[0].W, layers[0].b, layers[1].W, layers[1].b)
    for f, l in zip(feats, labels):
        m.utterance(f, l, bptt, lr, mmt, wc)
    err, frames, correct = obj.stats()
    assert frames == m.frames == tr.frames
    np.testing.assert_allclose(err, m.xent, rtol=1e-4)
    assert abs(correct - m.correct) <= 1  # argmax near-ties may flip on fp32 rounding
    Wr, br = net.recurrent_params(0)
    np.testing.assert_allclose(Wr, m.Wr, rtol=2e-3, atol=2e-5)
    np.testing.assert_allclose(br, m.br, rtol=2e-3, atol=2e-5)
    W2, b2 = net.linear_params()[0]
    np.testing.assert_allclose(W2, m.W2, rtol=2e-3, atol=2e-5)
    np.testing.assert_allclose(b2, m.b2, rtol=2e-3, atol=2e-5)


def _train_rnn(layers, feats, labels, bptt, lr, mmt, wc, generic, crossval=False):
    os.environ["TNET_RNN_GENERIC"] = "1" if generic else "0"
    try:
        net = Network.from_layers(layers)
        net.set_learn_rate(lr)
        net.set_momentum(mmt)
        net.set_weightcost(wc)
        obj = Objective()
        RnnTrainer(net, obj, bptt=bptt, crossval=crossval).train_corpus(feats, labels)
        return obj.stats(), net.recurrent_params(0), net.linear_params()[0]
    finally:
        os.environ.pop("TNET_RNN_GENERIC", None)


@pytest.mark.parametrize("S,bptt,mmt,wc", [(10, 4, 0.0, 0.0), (135, 2, 0.5, 1e-4), (4000, 4, 0.9, 0.0),
                                           (37, 0, 0.0, 1e-3), (135, 8, 0.0, 0.0)])
def test_rnn_fused_frame_matches_component_chain(S, bptt, mmt, wc):
    """the fused per-frame launch chain vs the component-by-component chain (Propagate, EvaluateLabels,
    Backpropagate + Update per layer) on the same utterances"""
    nIn, H, lr = 40, 64, 0.02
    rng = np.random.default_rng(S)
    layers = formats.gen_recurrent_init(nIn, H, S, seed=11)
    feats = [rng.standard_normal((T, nIn)).astype(np.float32) for T in (50, 33)]
    labels = [rng.integers(0, S, len(f)).astype(np.int32) for f in feats]
    labels[1][::9] = -1  # unlabeled frames: zero target
    a = _train_rnn(layers, feats, labels, bptt, lr, mmt, wc, generic=False)
    b = _train_rnn(layers, feats, labels, bptt, lr, mmt, wc, generic=True)
    (ea, fa, ca), (eb, fb, cb) = a[0], b[0]
    assert fa == fb == 83
    np.testing.assert_allclose(ea, eb, rtol=1e-5)
    assert abs(ca - cb) <= 1
    for x, y in zip(a[1] + a[2], b[1] + b[2]):
        np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("crossval", [False, True])
@pytest.mark.parametrize("S,bptt,mmt", [(135, 4, 0.0), (4000, 2, 0.5)])
def test_rnn_graph_replay_matches_eager(S, bptt, mmt, crossval):
    """the per-frame chain recorded once per utterance length and replayed as a hipGraph (default)
    vs the same chain launched eagerly (TNET_RNN_GRAPH=0): bit-identical statistics and weights.
    Lengths repeat (recorded on the second sighting, replayed from the third), interleave, and the
    learning rate changes between passes (a new key: recorded again)."""
    nIn, H = 40, 64
    rng = np.random.default_rng(S + bptt)
    layers = formats.gen_recurrent_init(nIn, H, S, seed=13)
    lens = [30, 30, 30, 21, 30, 21, 21, 30]
    feats = [rng.standard_normal((T, nIn)).astype(np.float32) for T in lens]
    labels = [rng.integers(0, S, T).astype(np.int32) for T in lens]

    def run(graph):
        os.environ["TNET_RNN_GRAPH"] = graph
        try:
            net = Network.from_layers(layers)
            net.set_momentum(mmt)
            obj = Objective()
            tr = RnnTrainer(net, obj, bptt=bptt, crossval=crossval)
            for lr in (0.02, 0.01):
                net.set_learn_rate(lr)
                tr.train_corpus(feats, labels)
            return obj.stats(), net.recurrent_params(0) + net.linear_params()[0]
        finally:
            os.environ.pop("TNET_RNN_GRAPH", None)

    (sa, pa), (sb, pb) = run("1"), run("0")
    assert sa == sb and sa[1] == 2 * sum(lens)
    for x, y in zip(pa, pb):
        np.testing.assert_array_equal(x, y)
    if crossval:  # cross-validation replays leave the weights as read
        np.testing.assert_array_equal(pa[0], layers[0].W)
        np.testing.assert_array_equal(pa[2], layers[1].W)


def test_rnn_fused_crossval_leaves_weights():
    nIn, H, S = 24, 32, 10
    rng = np.random.default_rng(5)
    layers = formats.gen_recurrent_init(nIn, H, S, seed=3)
    feats = [rng.standard_normal((40, nIn)).astype(np.float32)]
    labels = [rng.integers(0, S, 40).astype(np.int32)]
    (e, f, c), (Wr, br), (W2, b2) = _train_rnn(layers, feats, labels, 4, 0.05, 0.0, 0.0, False, crossval=True)
    (e2, f2, c2), _, _ = _train_rnn(layers, feats, labels, 4, 0.05, 0.0, 0.0, True, crossval=True)
    assert f == f2 == 40 and c == c2
    np.testing.assert_allclose(e, e2, rtol=1e-5)
    np.testing.assert_array_equal(Wr, layers[0].W)
    np.testing.assert_array_equal(W2, layers[1].W)


@pytest.mark.parametrize("K0,K1,N", [(440, 512, 512), (7, 0, 5), (0, 33, 70)])
def test_gemv_rowvec_cat_pushes_history_row(K0, K1, N):
    rng = np.random.default_rng(K0 + K1)
    v0, v1 = rng.standard_normal(max(K0, 1)).astype(np.float32), rng.standard_normal(max(K1, 1)).astype(np.float32)
    W = (0.05 * rng.standard_normal((K0 + K1, N))).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    d0, d1 = DeviceArray.vector(v0), DeviceArray.vector(v1)
    dW, db, y, hist = DeviceArray.from_numpy(W), DeviceArray.vector(b), DeviceArray(1, N), DeviceArray(1, K0 + K1)
    ws = DeviceArray(1, max(1, lib().tnet_gemv_workspace(K0 + K1, N) // 4))
    check(lib().tnet_gemv_rowvec_cat(d0.ptr, K0, d1.ptr, K1, hist.ptr, dW.ptr, dW.stride, db.ptr, y.ptr, N, 1,
                                     ws.ptr, S()))
    row = np.concatenate([v0[:K0], v1[:K1]])
    np.testing.assert_array_equal(hist.numpy().ravel(), row)
    a = b + row.astype(np.float64) @ W
    np.testing.assert_allclose(y.numpy().ravel(), 1 / (1 + np.exp(-a)), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("K,N,t", [(512, 135, 7), (512, 4000, 3999), (64, 1, 0), (100, 300, -1)])
def test_gemv_rowvec_softmax_xent(K, N, t):
    rng = np.random.default_rng(N)
    v = rng.standard_normal(K).astype(np.float32)
    W = (0.1 * rng.standard_normal((K, N))).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    dv, dW, db = DeviceArray.vector(v), DeviceArray.from_numpy(W), DeviceArray.vector(b)
    z, y, e = DeviceArray(1, N), DeviceArray(1, N), DeviceArray(1, N)
    lab = DeviceArray.vector(np.array([t], np.int32))
    stats = DeviceArray(1, 1024, np.float64, stride=1024)
    ws = DeviceArray(1, max(1, lib().tnet_gemv_workspace(K, N) // 4))
    check(lib().tnet_gemv_rowvec_softmax_xent(dv.ptr, K, dW.ptr, dW.stride, db.ptr, z.ptr, y.ptr, e.ptr, N, lab.ptr,
                                              stats.ptr, ws.ptr, S()))
    zr = b + v.astype(np.float64) @ W
    np.testing.assert_allclose(z.numpy().ravel(), zr, rtol=1e-5, atol=1e-5)
    Yr = orc.softmax(zr.reshape(1, -1).astype(np.float32))
    Er, xent, correct = orc.xent_eval(Yr, np.array([t], np.int32))
    np.testing.assert_allclose(y.numpy(), Yr, rtol=2e-5, atol=1e-9)
    np.testing.assert_allclose(e.numpy(), Er, rtol=2e-5, atol=1e-8)
    s = stats.numpy()[0]
    np.testing.assert_allclose(s[0::2].sum(), xent, rtol=1e-5, atol=1e-6)
    assert int(round(s[1::2].sum())) == correct
    ok = DeviceArray(1, 4097)
    assert lib().tnet_gemv_rowvec_softmax_xent(dv.ptr, K, ok.ptr, 4097, None, None, None, None, 4097, lab.ptr,
                                               None, ws.ptr, S()) == -4  # TNET_ERR_UNSUPPORTED: N > 4096


@pytest.mark.parametrize("mmt", [0.0, 0.9])
@pytest.mark.parametrize("n_in,n_out", [(512, 135), (512, 4000), (13, 7)])
def test_affine_bwd_update_row(mmt, n_in, n_out):
    """e_out = W e with the weights before the update, the update of tnet_affine_update_row, and the
    diff-sigmoid d = e_out s (1 - s)"""
    rng = np.random.default_rng(n_out)
    x, s = rng.random(n_in).astype(np.float32), rng.random(n_in).astype(np.float32)
    e = (0.1 * rng.standard_normal(n_out)).astype(np.float32)
    W, corr = (0.1 * rng.standard_normal((n_in, n_out))).astype(np.float32), rng.standard_normal((n_in, n_out)).astype(np.float32)
    b, cb = rng.standard_normal(n_out).astype(np.float32), rng.standard_normal(n_out).astype(np.float32)
    dx, ds, de, dW, db = (DeviceArray.vector(x), DeviceArray.vector(s), DeviceArray.vector(e),
                          DeviceArray.from_numpy(W), DeviceArray.vector(b))
    dC, dCb = DeviceArray.from_numpy(corr), DeviceArray.vector(cb)
    eo, d = DeviceArray(1, n_in), DeviceArray(1, n_in)
    scale, l2 = -0.02, -1e-4
    check(lib().tnet_affine_bwd_update_row(dx.ptr, n_in, de.ptr, n_out, dW.ptr, dW.stride, dC.ptr, dC.stride, db.ptr,
                                           dCb.ptr, scale, mmt, l2, eo.ptr, ds.ptr, d.ptr, S()))
    er = W.astype(np.float64) @ e
    np.testing.assert_allclose(eo.numpy().ravel(), er, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(d.numpy().ravel(), er * s * (1 - s), rtol=1e-5, atol=1e-6)
    c = np.outer(x, e).astype(np.float64) + (mmt * corr if mmt else 0)
    w = W + scale * c
    w = w + l2 * w
    np.testing.assert_allclose(dW.numpy(), w, rtol=1e-6, atol=1e-7)
    gb = e + mmt * cb if mmt else e.astype(np.float64)
    np.testing.assert_allclose(db.numpy().ravel(), b + scale * gb, rtol=1e-6, atol=1e-7)
    if mmt:
        np.testing.assert_allclose(dC.numpy(), c, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(dCb.numpy().ravel(), gb, rtol=1e-6, atol=1e-7)
    else:  # momentum 0: the correction buffers are not touched
        np.testing.assert_array_equal(dC.numpy(), corr)


@pytest.mark.parametrize("nIn,H,N,t", [(440, 512, 4000, 17), (440, 512, 135, 3), (30, 70, 300, -1), (8, 64, 5, 9)])
def test_rnn_output_chain_kernels(nIn, H, N, t):
    """tnet_gemv_rowvec_partial -> tnet_rnn_out_partial -> tnet_rnn_out_stats -> tnet_rnn_out_bwd_update
    (the fused frame's output side) vs numpy in fp64: h, z, the softmax error inside the SGD of Wo / bo,
    e_out = Wo e (old Wo), d = e_out h (1 - h), cross-entropy and the argmax key (rtol 1e-5)"""
    rng = np.random.default_rng(N + H)
    x = rng.standard_normal(nIn).astype(np.float32)
    yp = rng.random(H).astype(np.float32)
    W = (0.05 * rng.standard_normal((nIn + H, H))).astype(np.float32)
    b = rng.standard_normal(H).astype(np.float32)
    Wo = (0.05 * rng.standard_normal((H, N))).astype(np.float32)
    bo = rng.standard_normal(N).astype(np.float32)
    scale, l2 = -0.03, -1e-5
    d = {k: DeviceArray.from_numpy(v.reshape(1, -1) if v.ndim == 1 else v) for k, v in
         dict(x=x, yp=yp, W=W, b=b, Wo=Wo, bo=bo).items()}
    hs, os_, G = -(-(nIn + H) // 64), -(-H // 64), -(-N // 256)
    hpart, opart = DeviceArray(hs, H), DeviceArray(os_, N)
    hist, h, z = DeviceArray(1, nIn + H), DeviceArray(1, H), DeviceArray(1, N)
    smx = DeviceArray(1, 2 * G, np.float64, stride=2 * G)
    lab = DeviceArray.vector(np.array([t], np.int32))
    eo, dd, e, y = DeviceArray(1, H), DeviceArray(1, H), DeviceArray(1, N), DeviceArray(1, N)
    stats = DeviceArray(1, 1024, np.float64, stride=1024)
    key = DeviceArray.vector(np.zeros(2, np.int32))  # one 64-bit key
    check(lib().tnet_gemv_rowvec_partial(d["x"].ptr, nIn, d["yp"].ptr, H, hist.ptr, d["W"].ptr, d["W"].stride, H,
                                         hpart.ptr, S()))
    check(lib().tnet_rnn_out_partial(hpart.ptr, hs, d["b"].ptr, h.ptr, H, d["Wo"].ptr, d["Wo"].stride, N, opart.ptr,
                                     S()))
    check(lib().tnet_rnn_out_stats(opart.ptr, H, N, d["bo"].ptr, z.ptr, smx.ptr, S()))
    check(lib().tnet_rnn_out_bwd_update(z.ptr, smx.ptr, G, N, lab.ptr, h.ptr, H, d["Wo"].ptr, d["Wo"].stride, None, 0,
                                        d["bo"].ptr, None, scale, 0.0, l2, y.ptr, e.ptr, eo.ptr, dd.ptr, stats.ptr,
                                        key.ptr, 1, S()))
    v = np.concatenate([x, yp]).astype(np.float64)
    np.testing.assert_array_equal(hist.numpy().ravel(), np.concatenate([x, yp]))
    hr = 1 / (1 + np.exp(-(b + v @ W)))
    np.testing.assert_allclose(h.numpy().ravel(), hr, rtol=1e-5, atol=1e-6)
    zr = bo + hr @ Wo
    np.testing.assert_allclose(z.numpy().ravel(), zr, rtol=1e-5, atol=1e-5)
    yr = np.exp(zr - zr.max())
    yr /= yr.sum()
    tt = t if 0 <= t < N else -1
    er = yr - (np.arange(N) == tt)
    np.testing.assert_allclose(y.numpy().ravel(), yr, rtol=2e-5, atol=1e-9)
    np.testing.assert_allclose(e.numpy().ravel(), er, rtol=2e-5, atol=1e-8)
    eor = Wo.astype(np.float64) @ er
    np.testing.assert_allclose(eo.numpy().ravel(), eor, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(dd.numpy().ravel(), eor * hr * (1 - hr), rtol=1e-4, atol=1e-6)
    Wn = Wo + scale * np.outer(hr, er)
    np.testing.assert_allclose(d["Wo"].numpy(), Wn + l2 * Wn, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(d["bo"].numpy().ravel(), bo + scale * er, rtol=1e-5, atol=1e-7)
    xent = -np.log(max(yr[tt], 1.1754944e-38)) if tt >= 0 else 0.0
    np.testing.assert_allclose(stats.numpy()[0][0::2].sum(), xent, rtol=1e-5, atol=1e-6)
    k = int(key.numpy().ravel().view(np.uint64)[0])
    assert 0xFFFFFFFF - (k & 0xFFFFFFFF) == int(np.argmax(y.numpy().ravel()))
    # frame accuracy from the key
    st2 = DeviceArray(1, 1024, np.float64, stride=1024)
    check(lib().tnet_argmax_correct(key.ptr, lab.ptr, 1, N, st2.ptr, S()))
    assert st2.numpy()[0][1] == float(int(np.argmax(y.numpy().ravel())) == (tt if tt >= 0 else 0))


@pytest.mark.parametrize("nIn,H,N,t", [(440, 512, 4000, 17), (440, 512, 135, 3), (30, 70, 300, -1), (8, 64, 5, 9)])
def test_rnn_out_full(nIn, H, N, t):
    """tnet_rnn_out_full (the trainer's output side: h finished by every workgroup, complete z per 64
    columns, one softmax pair per 64 columns) -> tnet_rnn_out_bwd_update with ceil(N/64) pairs vs numpy
    in fp64 (the tolerances of test_rnn_output_chain_kernels)"""
    rng = np.random.default_rng(N + H + 1)
    x = rng.standard_normal(nIn).astype(np.float32)
    yp = rng.random(H).astype(np.float32)
    W = (0.05 * rng.standard_normal((nIn + H, H))).astype(np.float32)
    b = rng.standard_normal(H).astype(np.float32)
    Wo = (0.05 * rng.standard_normal((H, N))).astype(np.float32)
    bo = rng.standard_normal(N).astype(np.float32)
    scale, l2 = -0.03, -1e-5
    d = {k: DeviceArray.from_numpy(v.reshape(1, -1) if v.ndim == 1 else v) for k, v in
         dict(x=x, yp=yp, W=W, b=b, Wo=Wo, bo=bo).items()}
    hs, G = -(-(nIn + H) // 64), -(-N // 64)
    hpart = DeviceArray(hs, H)
    hist, h, z = DeviceArray(1, nIn + H), DeviceArray(1, H), DeviceArray(1, N)
    smx = DeviceArray(1, 2 * G, np.float64, stride=2 * G)
    lab = DeviceArray.vector(np.array([t], np.int32))
    eo, dd, e, y = DeviceArray(1, H), DeviceArray(1, H), DeviceArray(1, N), DeviceArray(1, N)
    stats = DeviceArray(1, 1024, np.float64, stride=1024)
    key = DeviceArray.vector(np.zeros(2, np.int32))
    check(lib().tnet_gemv_rowvec_partial(d["x"].ptr, nIn, d["yp"].ptr, H, hist.ptr, d["W"].ptr, d["W"].stride, H,
                                         hpart.ptr, S()))
    check(lib().tnet_rnn_out_full(hpart.ptr, hs, d["b"].ptr, h.ptr, H, d["Wo"].ptr, d["Wo"].stride, N, d["bo"].ptr,
                                  z.ptr, smx.ptr, S()))
    check(lib().tnet_rnn_out_bwd_update(z.ptr, smx.ptr, G, N, lab.ptr, h.ptr, H, d["Wo"].ptr, d["Wo"].stride, None, 0,
                                        d["bo"].ptr, None, scale, 0.0, l2, y.ptr, e.ptr, eo.ptr, dd.ptr, stats.ptr,
                                        key.ptr, 1, S()))
    v = np.concatenate([x, yp]).astype(np.float64)
    hr = 1 / (1 + np.exp(-(b + v @ W)))
    np.testing.assert_allclose(h.numpy().ravel(), hr, rtol=1e-5, atol=1e-6)
    zr = bo + hr @ Wo
    np.testing.assert_allclose(z.numpy().ravel(), zr, rtol=1e-5, atol=1e-5)
    yr = np.exp(zr - zr.max())
    yr /= yr.sum()
    tt = t if 0 <= t < N else -1
    er = yr - (np.arange(N) == tt)
    np.testing.assert_allclose(y.numpy().ravel(), yr, rtol=2e-5, atol=1e-9)
    np.testing.assert_allclose(e.numpy().ravel(), er, rtol=2e-5, atol=1e-8)
    eor = Wo.astype(np.float64) @ er
    np.testing.assert_allclose(eo.numpy().ravel(), eor, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(dd.numpy().ravel(), eor * hr * (1 - hr), rtol=1e-4, atol=1e-6)
    Wn = Wo + scale * np.outer(hr, er)
    np.testing.assert_allclose(d["Wo"].numpy(), Wn + l2 * Wn, rtol=1e-5, atol=1e-7)
    xent = -np.log(max(yr[tt], 1.1754944e-38)) if tt >= 0 else 0.0
    np.testing.assert_allclose(stats.numpy()[0][0::2].sum(), xent, rtol=1e-5, atol=1e-6)
    k = int(key.numpy().ravel().view(np.uint64)[0])
    assert 0xFFFFFFFF - (k & 0xFFFFFFFF) == int(np.argmax(y.numpy().ravel()))


@pytest.mark.parametrize("nIn,H,steps,R,head,mmt,wc", [(440, 512, 5, 6, 2, 0.0, 0.0), (440, 512, 5, 6, 5, 0.5, 1e-4),
                                                      (30, 70, 3, 4, 0, 0.9, 1e-3), (8, 64, 1, 2, 1, 0.0, 0.0),
                                                      (100, 200, 9, 10, 7, 0.5, 1e-4)])
def test_gemv_rowvec_partial_update(nIn, H, steps, R, head, mmt, wc):
    """tnet_gemv_rowvec_partial_update (the previous frame's recurrent update folded into the next
    frame's forward) = tnet_rnn_update then tnet_gemv_rowvec_partial: W, b, corr_b, the partials and the
    pushed history row bit-identical (same per-element arithmetic and order); the push lands on the ring
    row the update does not read; steps > 9 or steps >= R are refused (TNET_ERR_UNSUPPORTED: the trainer
    then runs the update on its own)"""
    rng = np.random.default_rng(H + steps)
    K = nIn + H
    W = (0.05 * rng.standard_normal((K, H))).astype(np.float32)
    b = rng.standard_normal(H).astype(np.float32)
    cb = (0.01 * rng.standard_normal(H)).astype(np.float32)
    hist = rng.standard_normal((R, K)).astype(np.float32)
    D = (0.1 * rng.standard_normal((steps, H))).astype(np.float32)
    x = rng.standard_normal(nIn).astype(np.float32)
    yp = rng.random(H).astype(np.float32)
    lr = 0.02
    push = (head + R - 1) % R
    outs = []
    for fused in (False, True):
        dW, db, dcb, dh, dD = (DeviceArray.from_numpy(W), DeviceArray.vector(b), DeviceArray.vector(cb),
                               DeviceArray.from_numpy(hist), DeviceArray.from_numpy(D))
        dx, dy = DeviceArray.vector(x), DeviceArray.vector(yp)
        part = DeviceArray(-(-K // 64), H)
        row = dh.ptr + push * dh.stride * 4
        if fused:
            check(lib().tnet_gemv_rowvec_partial_update(dx.ptr, nIn, dy.ptr, H, row, dW.ptr, dW.stride, H, part.ptr,
                                                        dh.ptr, dh.stride, head, R, dD.ptr, dD.stride, steps, db.ptr,
                                                        dcb.ptr, lr, mmt, wc, S()))
        else:
            check(lib().tnet_rnn_update(dW.ptr, dW.stride, K, H, dh.ptr, dh.stride, head, R, dD.ptr, dD.stride, steps,
                                        db.ptr, dcb.ptr, lr, mmt, wc, S()))
            check(lib().tnet_gemv_rowvec_partial(dx.ptr, nIn, dy.ptr, H, row, dW.ptr, dW.stride, H, part.ptr, S()))
        synchronize()
        outs.append([a.numpy() for a in (dW, db, dcb, part, dh)])
    for a, c in zip(*outs):
        np.testing.assert_array_equal(a, c)
    np.testing.assert_array_equal(outs[1][4][push], np.concatenate([x, yp]))
    dummy = DeviceArray(4, 64)
    assert lib().tnet_gemv_rowvec_partial_update(dummy.ptr, 8, dummy.ptr, 8, None, dummy.ptr, 64, 8, dummy.ptr,
                                                 dummy.ptr, 64, 0, 4, dummy.ptr, 64, 4, dummy.ptr, dummy.ptr, lr,
                                                 mmt, wc, S()) != 0
