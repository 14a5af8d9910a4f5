"""Recurrent path (BASELINE config 5: Elman RNN trained frame by frame with truncated BPTT, the
TRecurrentCu loop) on the GPU vs the oracle's restatement of CuRecurrent / TRecurrentCu.

CuRecurrent is CUDA-only in the reference (no CPU counterpart), so parity is against the
restatement (oracle/tnet_oracle.c orc_rnn_utterance) -- "parity restated", not reference-run.
Tolerances: single-frame kernels rtol 1e-5; after whole utterances (hundreds of sequential
per-frame SGD updates, each amplifying fp32 rounding differences) parameters rtol 2e-3 /
atol 2e-5 and summed cross-entropy rtol 1e-4.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle as orc  # noqa: E402
from tnet_amd import DeviceArray, Network, Objective, RnnTrainer, formats  # noqa: E402
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
    """Two utterances through TRecurrentCu semantics (history reset per utterance)."""
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
    Wr, br = net.recurrent_params(0)
    np.testing.assert_allclose(Wr, m.Wr, rtol=2e-3, atol=2e-5)
    np.testing.assert_allclose(br, m.br, rtol=2e-3, atol=2e-5)
    W2, b2 = net.linear_params()[0]
    np.testing.assert_allclose(W2, m.W2, rtol=2e-3, atol=2e-5)
    np.testing.assert_allclose(b2, m.b2, rtol=2e-3, atol=2e-5)
