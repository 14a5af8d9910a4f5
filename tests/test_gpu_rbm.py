"""RBM pre-training path (BASELINE config 4: Gauss-Bernoulli RBM, CD-1) on the GPU vs the oracle's
restatement of CuRand / CuRbm / TRbmCu.

The reference RBM code is CUDA-only (no CPU counterpart in TNetLib), so parity is against the
restatement (oracle/tnet_oracle.c: orc_rand_*, orc_rbm_step) -- "parity restated", not
reference-run.  Tolerances:
  uniforms, binarised states, generator state: bit-exact (integer recurrences + one double->float
  rounding, identical by construction);
  Box-Muller normals: abs 2e-5 (logf/sinf ulp differences between libm and the device);
  per-step / per-epoch parameters: rtol 2e-4, atol 2e-6 (fp32 GEMM order; the fused update sums
  positive and negative statistics in one GEMM where the reference runs two);
  reconstruction MSE over an epoch: rtol 1e-4.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle as orc  # noqa: E402
from tnet_amd import DeviceArray, Network, RbmTrainer, formats  # noqa: E402
from tnet_amd._lib import MatrixDim, check, lib  # noqa: E402


def S():
    return lib().tnet_stream()


def _state_dev(rs, rows, cols):
    return [DeviceArray.from_numpy(z.reshape(rows, cols)) for z in rs.z]


@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 70), (64, 128), (17, 300)])
def test_rand_uniform_bitexact(rows, cols):
    rs = orc.RandState(1234, rows, cols)
    z = _state_dev(rs, rows, cols)
    out = DeviceArray(rows, cols)
    for _ in range(3):
        check(lib().tnetF_rand(out.ptr, out.dim, *[a.ptr for a in z], S()))
        np.testing.assert_array_equal(out.numpy(), rs.uniform())
    for a, b in zip(z, rs.z):
        np.testing.assert_array_equal(a.numpy().reshape(-1), b)


def test_gauss_rand_and_noise():
    rows, cols = 32, 96
    rs = orc.RandState(77, rows, cols)
    z = _state_dev(rs, rows, cols)
    out = DeviceArray(rows, cols)
    check(lib().tnetF_gauss_rand(out.ptr, out.dim, *[a.ptr for a in z], S()))
    np.testing.assert_allclose(out.numpy(), rs.gauss(), rtol=0, atol=2e-5)
    base = np.random.default_rng(0).standard_normal((rows, cols)).astype(np.float32)
    tgt = DeviceArray.from_numpy(base)
    check(lib().tnet_add_gauss_noise(tgt.ptr, tgt.dim, 0.5, *[a.ptr for a in z], S()))
    np.testing.assert_allclose(tgt.numpy(), base + 0.5 * rs.gauss(), rtol=0, atol=2e-5)
    for a, b in zip(z, rs.z):
        np.testing.assert_array_equal(a.numpy().reshape(-1), b)


def test_rand_binarize_bitexact():
    rows, cols = 48, 200
    rs = orc.RandState(9, rows, cols)
    z = _state_dev(rs, rows, cols)
    P = np.random.default_rng(3).random((rows, cols)).astype(np.float32)
    dP = DeviceArray.from_numpy(P)
    st = DeviceArray(rows, cols)
    check(lib().tnet_rand_binarize(st.ptr, st.stride, dP.ptr, dP.dim, *[a.ptr for a in z], S()))
    np.testing.assert_array_equal(st.numpy(), (P > rs.uniform()).astype(np.float32))
    # the unfused reference form: uniforms then _binarize_probs
    U = DeviceArray(rows, cols)
    check(lib().tnetF_rand(U.ptr, U.dim, *[a.ptr for a in z], S()))
    st2 = DeviceArray(rows, cols)
    check(lib().tnetF_binarize_probs(st2.ptr, dP.ptr, U.ptr, dP.dim, S()))
    np.testing.assert_array_equal(st2.numpy(), (P > rs.uniform()).astype(np.float32))


@pytest.mark.parametrize("cfg", ["auto", "g64x64k32s4w4", "m64x128k64s2"])
@pytest.mark.parametrize("rows,V,H", [(256, 440, 2048), (1024, 440, 2048), (33, 37, 70), (1, 5, 3)])
def test_affine_fwd_sample_matches_two_launches(rows, V, H, cfg):
    """positive phase + HybridTaus binarisation in one launch: probabilities, sampled states and the
    advanced generator states bit-identical to tnet_affine_fwd(act 1) + tnet_rand_binarize, and the
    states equal to the oracle's draws"""
    rng = np.random.default_rng(rows + V)
    X = rng.standard_normal((rows, V)).astype(np.float32)
    W = (0.05 * rng.standard_normal((V, H))).astype(np.float32)
    b = rng.standard_normal(H).astype(np.float32)
    dX, dW, db = DeviceArray.from_numpy(X), DeviceArray.from_numpy(W), DeviceArray.vector(b)
    check(lib().tnet_gemm_config(cfg.encode()))
    try:
        out = []
        for fused in (True, False):
            rs = orc.RandState(31, rows, H)
            z = _state_dev(rs, rows, H)
            Y, st = DeviceArray(rows, H), DeviceArray(rows, H)
            if fused:
                check(lib().tnet_affine_fwd_sample(dX.ptr, dX.dim, dW.ptr, dW.dim, db.ptr, Y.ptr, Y.dim, st.ptr,
                                                   st.stride, *[a.ptr for a in z], S()))
            else:
                check(lib().tnet_affine_fwd(dX.ptr, dX.dim, dW.ptr, dW.dim, db.ptr, Y.ptr, Y.dim, 1, S()))
                check(lib().tnet_rand_binarize(st.ptr, st.stride, Y.ptr, Y.dim, *[a.ptr for a in z], S()))
            out.append((Y.numpy(), st.numpy(), [a.numpy() for a in z]))
            if fused:
                np.testing.assert_array_equal(st.numpy(), (Y.numpy() > rs.uniform()).astype(np.float32))
                for a, zb in zip(z, rs.z):
                    np.testing.assert_array_equal(a.numpy().reshape(-1), zb)
    finally:
        check(lib().tnet_gemm_config(b"auto"))
    (Y1, s1, z1), (Y2, s2, z2) = out
    np.testing.assert_array_equal(Y1, Y2)
    np.testing.assert_array_equal(s1, s2)
    for a, b2 in zip(z1, z2):
        np.testing.assert_array_equal(a, b2)


@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_affine_fwd_negated_and_transposed(act):
    rng = np.random.default_rng(act)
    X = rng.standard_normal((70, 40)).astype(np.float32)
    W = (0.1 * rng.standard_normal((40, 90))).astype(np.float32)
    b = rng.standard_normal(90).astype(np.float32)
    dX, dW, db = DeviceArray.from_numpy(X), DeviceArray.from_numpy(W), DeviceArray.vector(b)
    Y = DeviceArray(70, 90)
    check(lib().tnet_affine_fwd(dX.ptr, dX.dim, dW.ptr, dW.dim, db.ptr, Y.ptr, Y.dim, act, S()))
    a = X.astype(np.float64) @ W + b
    ref = {0: a, 1: 1 / (1 + np.exp(-a)), 2: -a, 3: -1 / (1 + np.exp(-a))}[act]
    np.testing.assert_allclose(Y.numpy(), ref, rtol=1e-5, atol=1e-5)
    if act < 2:  # reconstruction: X2 [70 x 90] W^T + vb
        X2 = rng.standard_normal((70, 90)).astype(np.float32)
        vb = rng.standard_normal(40).astype(np.float32)
        dX2, dvb = DeviceArray.from_numpy(X2), DeviceArray.vector(vb)
        Y2 = DeviceArray(70, 40)
        check(lib().tnet_affine_fwd_t(dX2.ptr, dX2.dim, dW.ptr, dW.dim, dvb.ptr, Y2.ptr, Y2.dim, act, S()))
        a2 = X2.astype(np.float64) @ W.T + vb
        np.testing.assert_allclose(Y2.numpy(), a2 if act == 0 else 1 / (1 + np.exp(-a2)), rtol=1e-5, atol=1e-5)


def _cd1_reference(W, vb, hb, cW, cvb, chb, pv, ph, nv, nh, lr, mmt, wc):
    N = pv.shape[0]
    cW = (-lr / N) * (nv.T.astype(np.float64) @ nh) + mmt * cW
    cW = (lr / N) * (pv.T.astype(np.float64) @ ph) + cW
    cW = (-lr * wc) * W + cW
    W = W + cW
    cvb = (-lr / N) * nv.sum(0, dtype=np.float64) + mmt * cvb + (lr / N) * pv.sum(0, dtype=np.float64)
    chb = (-lr / N) * nh.sum(0, dtype=np.float64) + mmt * chb + (lr / N) * ph.sum(0, dtype=np.float64)
    return W, vb + cvb, hb + chb, cW, cvb, chb


@pytest.mark.parametrize("V,H,B", [(40, 64, 32), (440, 256, 64), (33, 70, 17)])
def test_rbm_update_generic_and_stacked(V, H, B):
    rng = np.random.default_rng(V + H)
    L = formats.gen_rbm_init(V, H, seed=4)[0]
    pv, nv = (rng.standard_normal((B, V)).astype(np.float32) for _ in range(2))
    ph, nh = (rng.random((B, H)).astype(np.float32) for _ in range(2))
    lr, mmt, wc = 0.1, 0.5, 0.0002
    cW0 = (0.01 * rng.standard_normal((V, H))).astype(np.float32)
    cvb0 = (0.01 * rng.standard_normal(V)).astype(np.float32)
    chb0 = (0.01 * rng.standard_normal(H)).astype(np.float32)
    ref = _cd1_reference(L.W, L.extra["vis_bias"], L.b, cW0, cvb0, chb0, pv, ph, nv, nh, lr, mmt, wc)
    # generic CuRbm::RbmUpdate (two GEMMs + AddScaled, the reference's sequence), from zero momentum
    net = Network.from_layers([L])
    net.set_learn_rate(lr)
    net.set_momentum(mmt)
    net.set_weightcost(wc)
    ref0 = _cd1_reference(L.W, L.extra["vis_bias"], L.b, 0 * cW0, 0 * cvb0, 0 * chb0, pv, ph, nv, nh, lr, mmt, wc)
    net.rbm_update(0, *(DeviceArray.from_numpy(a) for a in (pv, ph, nv, nh)))
    W, vb, hb, _ = net.rbm_params(0)
    for got, want in zip((W, vb, hb), ref0[:3]):
        np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-6)
    # stacked one-GEMM form with momentum state
    dV = DeviceArray.from_numpy(np.concatenate([pv, nv]))
    dH = DeviceArray.from_numpy(np.concatenate([ph, -nh]))
    dW = DeviceArray.from_numpy(L.W)
    dc = DeviceArray.from_numpy(cW0)
    dvb, dhb = DeviceArray.vector(L.extra["vis_bias"]), DeviceArray.vector(L.b)
    dcvb, dchb = DeviceArray.vector(cvb0), DeviceArray.vector(chb0)
    check(lib().tnet_rbm_update(dV.ptr, dV.dim, dH.ptr, dH.dim, dW.ptr, dW.dim, dc.ptr, dc.stride, lr / B, mmt,
                                -lr * wc, S()))
    check(lib().tnet_rbm_bias_update(dV.ptr, dV.dim, B, dvb.ptr, dcvb.ptr, lr / B, mmt, None, S()))
    check(lib().tnet_rbm_bias_update(dH.ptr, dH.dim, 2 * B, dhb.ptr, dchb.ptr, lr / B, mmt, None, S()))
    for got, want in zip((dW.numpy(), dvb.numpy().reshape(-1), dhb.numpy().reshape(-1), dc.numpy()),
                         (ref[0], ref[1], ref[2], ref[3])):
        np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-6)


@pytest.mark.parametrize("V,H,B", [(440, 2048, 256), (33, 70, 17), (64, 130, 600), (440, 200, 1024), (8, 40, 4096)])
def test_rbm_stats_update_matches_two_colsums_and_mse(V, H, B):
    """the one-launch bias updates + reconstruction MSE == two tnet_rbm_bias_update launches (bit
    for bit: same slab sums, same fp64 combine) + tnet_mse (fp64 sums, rtol 1e-12)"""
    rng = np.random.default_rng(V + B)
    Vs = rng.standard_normal((2 * B, V)).astype(np.float32)
    Hs = rng.random((2 * B, H)).astype(np.float32)
    Hs[B:] *= -1
    vb, hb = (rng.standard_normal(n).astype(np.float32) for n in (V, H))
    cvb, chb = (0.01 * rng.standard_normal(n).astype(np.float32) for n in (V, H))
    lr, mmt = 0.1, 0.5
    dV, dH = DeviceArray.from_numpy(Vs), DeviceArray.from_numpy(Hs)
    out = []
    for fused in (True, False):
        d = [DeviceArray.vector(a) for a in (vb, cvb, hb, chb)]
        st = DeviceArray(1, 1024, np.float64, stride=1024)
        if fused:
            check(lib().tnet_rbm_stats_update(dV.ptr, dV.dim, dH.ptr, dH.dim, B, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr,
                                              lr / B, mmt, st.ptr, S()))
        else:
            check(lib().tnet_rbm_bias_update(dV.ptr, dV.dim, B, d[0].ptr, d[1].ptr, lr / B, mmt, None, S()))
            check(lib().tnet_rbm_bias_update(dH.ptr, dH.dim, 2 * B, d[2].ptr, d[3].ptr, lr / B, mmt, None, S()))
            neg = DeviceArray.from_numpy(Vs[B:])
            pos = DeviceArray.from_numpy(Vs[:B])
            check(lib().tnet_mse(neg.ptr, neg.dim, pos.ptr, pos.stride, None, 0, st.ptr, S()))
        out.append(([a.numpy().reshape(-1) for a in d], st.numpy()[0][0::2].sum()))
    for a, b in zip(out[0][0], out[1][0]):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_allclose(out[0][1], out[1][1], rtol=1e-12)
    e = (Vs[B:] - Vs[:B]).astype(np.float64)
    np.testing.assert_allclose(out[0][1], (e * e).sum(), rtol=1e-6)


def test_rbm_text_round_trip(tmp_path):
    layers = formats.gen_rbm_init(24, 40, seed=2, vis_type="gauss", hid_type="bern")
    net = Network.from_layers(layers)
    assert net.components() == [("<rbm>", 24, 40)]
    W, vb, hb, types = net.rbm_params(0)
    assert types == ("gauss", "bern")
    np.testing.assert_array_equal(W, layers[0].W)
    np.testing.assert_array_equal(vb, layers[0].extra["vis_bias"])
    np.testing.assert_array_equal(hb, layers[0].b)
    p = str(tmp_path / "rbm.nnet")
    net.write(p)
    back = formats.read_nnet(p)
    assert back[0].tag == "<rbm>" and back[0].extra["vis_type"] == "gauss" and back[0].extra["hid_type"] == "bern"
    np.testing.assert_allclose(back[0].W, layers[0].W, rtol=1e-5, atol=1e-7)


def _rbm_epoch_expected(layer, corpus_feats, bunch, cache, seed, lr, mmt, wc):
    rs = orc.RandState(seed, bunch, layer.n_out)
    X = np.concatenate(corpus_feats)
    sched = orc.epoch_schedule_x([len(f) for f in corpus_feats], cache, bunch, rs.x_after)
    m = orc.RBM.from_layer(layer)
    for b in sched:
        m.step(X[b], rs, lr, mmt, wc)
    return m, len(sched)


@pytest.mark.parametrize("vis,hid", [("gauss", "bern"), ("bern", "bern"), ("gauss", "gauss")])
def test_rbm_trainer_epoch_matches_oracle(vis, hid):
    """TRbmCu epoch: cache fill/shuffle (after the CuRand seeds on the same lrand48 stream),
    CD-1 per bunch, reconstruction MSE -- config 4 in miniature (Gauss-Bernoulli first)."""
    V, H, B, cache, seed = 40, 64, 32, 256, 321
    lr, mmt, wc = 0.01, 0.5, 0.0002
    rng = np.random.default_rng(5)
    feats = [rng.standard_normal((int(n), V)).astype(np.float32) for n in rng.integers(40, 200, size=12)]
    if vis == "bern":
        feats = [1 / (1 + np.exp(-f)) for f in feats]
    layer = formats.round_trip_text(formats.gen_rbm_init(V, H, seed=6, vis_type=vis, hid_type=hid), 9)[0]
    net = Network.from_layers([layer])
    tr = RbmTrainer(net, bunchsize=B, cachesize=cache, seed=seed, learn_rate=lr, momentum=mmt, weightcost=wc)
    tr.train_corpus(feats)
    exp, nb = _rbm_epoch_expected(layer, feats, B, cache, seed, lr, mmt, wc)
    assert tr.steps == nb
    mse, frames = tr.stats()
    assert frames == exp.frames
    np.testing.assert_allclose(mse, exp.mse, rtol=1e-4)
    W, vb, hb, _ = net.rbm_params(0)
    np.testing.assert_allclose(W, exp.W, rtol=2e-4, atol=2e-6)
    np.testing.assert_allclose(vb, exp.vb, rtol=2e-4, atol=2e-6)
    np.testing.assert_allclose(hb, exp.hb, rtol=2e-4, atol=2e-6)
    rep = tr.report()
    assert rep.startswith("Mse:") and f"frames:{frames}" in rep


@pytest.mark.parametrize("V,H,B", [(440, 2048, 256), (33, 70, 17), (440, 2048, 1024), (64, 130, 600)])
def test_rbm_update_stats_one_launch_matches_two_calls(V, H, B):
    """tnet_rbm_update_stats (the CD-1 weight update and the statistics blocks in ONE launch) gives exactly
    what tnet_rbm_update + tnet_rbm_stats_update give (same tile bodies, same statistics blocks): W, its
    momentum, both biases and their momenta bit for bit, the MSE statistics equal; or declines with
    TNET_ERR_UNSUPPORTED where the update would run another configuration"""
    rng = np.random.default_rng(V * 7 + B)
    Vs = rng.standard_normal((2 * B, V)).astype(np.float32)
    Vs[B:] *= -1
    Hs = rng.random((2 * B, H)).astype(np.float32)
    Hs[B:] *= -1
    W0 = (0.05 * rng.standard_normal((V, H))).astype(np.float32)
    cW0 = (0.01 * rng.standard_normal((V, H))).astype(np.float32)
    vb, hb = (rng.standard_normal(n).astype(np.float32) for n in (V, H))
    cvb, chb = (0.01 * rng.standard_normal(n).astype(np.float32) for n in (V, H))
    lr, mmt, wc = 0.1, 0.5, 2e-4
    dV, dH = DeviceArray.from_numpy(Vs), DeviceArray.from_numpy(Hs)
    out = []
    for one in (True, False):
        dW, dc = DeviceArray.from_numpy(W0), DeviceArray.from_numpy(cW0)
        d = [DeviceArray.vector(a) for a in (vb, cvb, hb, chb)]
        st = DeviceArray(1, 1024, np.float64, stride=1024)
        if one:
            rc = lib().tnet_rbm_update_stats(dV.ptr, dV.dim, dH.ptr, dH.dim, dW.ptr, dW.dim, dc.ptr, dc.stride, lr / B,
                                             mmt, -lr * wc, B, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, st.ptr, S())
            if rc == -4:  # TNET_ERR_UNSUPPORTED: the trainer makes the two calls
                return
            check(rc)
        else:
            check(lib().tnet_rbm_update(dV.ptr, dV.dim, dH.ptr, dH.dim, dW.ptr, dW.dim, dc.ptr, dc.stride, lr / B, mmt,
                                        -lr * wc, S()))
            check(lib().tnet_rbm_stats_update(dV.ptr, dV.dim, dH.ptr, dH.dim, B, d[0].ptr, d[1].ptr, d[2].ptr,
                                              d[3].ptr, lr / B, mmt, st.ptr, S()))
        out.append(([dW.numpy(), dc.numpy()] + [a.numpy().reshape(-1) for a in d], st.numpy()[0][0::2]))
    for a, b in zip(out[0][0], out[1][0]):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_allclose(out[0][1].sum(), out[1][1].sum(), rtol=1e-12)


@pytest.mark.parametrize("V,H,B", [(440, 2048, 256), (33, 70, 17), (440, 2048, 1024)])
def test_rbm_update_stats_gather_matches_separate_calls(V, H, B):
    """tnet_rbm_update_stats_gather (the CD-1 update, its statistics and the NEXT bunch's visible rows in ONE
    launch) against tnet_rbm_update_stats + tnet_gather_bunch: W, momentum, biases, their momenta bit for bit,
    the MSE statistics equal, the gathered rows and ids exact; TNET_ERR_UNSUPPORTED where the update would
    run another configuration; TNET_ERR_ARG when the destination overlaps the statistics it reads"""
    rng = np.random.default_rng(V * 11 + B)
    Vs = rng.standard_normal((2 * B, V)).astype(np.float32)
    Vs[B:] *= -1
    Hs = rng.random((2 * B, H)).astype(np.float32)
    Hs[B:] *= -1
    W0 = (0.05 * rng.standard_normal((V, H))).astype(np.float32)
    cW0 = (0.01 * rng.standard_normal((V, H))).astype(np.float32)
    vb, hb = (rng.standard_normal(n).astype(np.float32) for n in (V, H))
    cvb, chb = (0.01 * rng.standard_normal(n).astype(np.float32) for n in (V, H))
    cache = rng.standard_normal((3 * B + 5, V)).astype(np.float32)
    perm = rng.permutation(cache.shape[0]).astype(np.int32)[:B]
    lab = np.zeros(cache.shape[0], np.int32)
    lr, mmt, wc = 0.1, 0.5, 2e-4
    dV, dH = DeviceArray.from_numpy(Vs), DeviceArray.from_numpy(Hs)
    dC, dL, dP = DeviceArray.from_numpy(cache), DeviceArray.vector(lab), DeviceArray.vector(perm)
    out = []
    for one in (True, False):
        dW, dc = DeviceArray.from_numpy(W0), DeviceArray.from_numpy(cW0)
        d = [DeviceArray.vector(a) for a in (vb, cvb, hb, chb)]
        st = DeviceArray(1, 1024, np.float64, stride=1024)
        dY = DeviceArray.from_numpy(np.full((B, V), np.nan, np.float32))
        dLo = DeviceArray.vector(np.full(B, 5, np.int32))
        head = [dV.ptr, dV.dim, dH.ptr, dH.dim, dW.ptr, dW.dim, dc.ptr, dc.stride, lr / B, mmt, -lr * wc, B, d[0].ptr,
                d[1].ptr, d[2].ptr, d[3].ptr, st.ptr]
        gargs = [dY.ptr, dC.ptr, dLo.ptr, dL.ptr, dP.ptr, dY.dim, dC.dim]
        if one:
            # the destination inside V: refused
            vview = MatrixDim(B, V, dV.stride)
            assert lib().tnet_rbm_update_stats_gather(*head, dV.ptr, dC.ptr, dLo.ptr, dL.ptr, dP.ptr, vview, dC.dim,
                                                      S()) == -1
            rc = lib().tnet_rbm_update_stats_gather(*head, *gargs, S())
            if rc == -4:
                assert lib().tnet_rbm_update_stats(*head, S()) == -4
                return
            check(rc)
        else:
            check(lib().tnet_rbm_update_stats(*head, S()))
            check(lib().tnet_gather_bunch(*gargs, S()))
        out.append(([dW.numpy(), dc.numpy()] + [a.numpy().reshape(-1) for a in d], st.numpy()[0][0::2],
                    dY.numpy(), dLo.numpy()[:, 0]))
    for a, b in zip(out[0][0], out[1][0]):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_allclose(out[0][1].sum(), out[1][1].sum(), rtol=1e-12)
    for k in (0, 1):
        np.testing.assert_array_equal(out[k][2], cache[perm])
        np.testing.assert_array_equal(out[k][3], lab[perm])
