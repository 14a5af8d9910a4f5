"""The backward GEMM from a transposed weight shadow (include/tnet_kernels.h tnet_affine_bwd_colsum_t,
tnet_affine_bwd_colsum_slabs_t, tnet_affine_update_bwd_pair_t, tnet_weight_shadow, tnet_transpose; the reference's
backward is CuBiasedLinearity::BackpropagateFnc, cuBiasedLinearity.cc:21-25, E_in = E W^T, and its update
cuBiasedLinearity.cc:46-64).

Tolerances: the error Eo = (E Wt) .* y (1 - y) is BIT-IDENTICAL to the NT form's (the same MFMA operands in the same
order per element -- the kernels' lane -> k map does not depend on the operand layout); the slab column sums add the
same fp32 rows in another order: |P - P_nt| <= 32 * 1.2e-7 * slab_sums(|Eo|) + 1e-7.  The shadow an update writes is
the updated W exactly (Wt == W^T bit for bit), for every 16x16 form (the 2048^2 128x128 direct update, the top
layer's 128x256 one, the 64x64 small forms, the update + backward pair, the mixed update + gather launch)."""
import numpy as np
import pytest

from tnet_amd import DeviceArray, synchronize
from tnet_amd._lib import check, lib

pytestmark = pytest.mark.gpu

TNET_ERR_UNSUPPORTED = -4


def S():
    return lib().tnet_stream()


def rnd(shape, seed, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)


def slab_sums(M, slab=32):
    n = -(-M.shape[0] // slab)
    return np.stack([M[s * slab:(s + 1) * slab].astype(np.float64).sum(0) for s in range(n)])


def transposed(dW):
    """Wt = W^T on the device (tnet_transpose)"""
    W = dW.numpy()
    dT = DeviceArray.from_numpy(np.full((W.shape[1], W.shape[0]), np.nan, np.float32))
    check(lib().tnet_transpose(dW.ptr, dW.dim, dT.ptr, dT.stride, S()))
    return dT


@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 70), (64, 64), (2048, 2048), (2048, 4000), (598, 1024), (65, 129)])
def test_transpose(rows, cols):
    W = rnd((rows, cols), 1)
    dT = transposed(DeviceArray.from_numpy(W))
    np.testing.assert_array_equal(dT.numpy(), W.T)


@pytest.mark.parametrize("rows,n_in,n_out", [(1024, 2048, 2048), (1024, 2048, 4000), (1024, 1024, 135),
                                             (256, 512, 1000), (96, 128, 64), (1000, 2048, 2048)])
def test_bwd_colsum_t_matches_nt(rows, n_in, n_out):
    """Eo from the shadow equals the NT form's bit for bit; the slab sums within fp32 reordering"""
    E, W = rnd((rows, n_out), 2, 0.01), rnd((n_in, n_out), 3, 0.1)
    Yb = (1 / (1 + np.exp(-rnd((rows, n_in), 4)))).astype(np.float32)
    dE, dW, dY = DeviceArray.from_numpy(E), DeviceArray.from_numpy(W), DeviceArray.from_numpy(Yb)
    dT = transposed(dW)
    slabs = lib().tnet_colsum_slabs(rows)
    out = {}
    for form in ("nt", "t"):
        dO = DeviceArray.from_numpy(np.full((rows, n_in), np.nan, np.float32))
        dP = DeviceArray.from_numpy(np.full((slabs, n_in), np.nan, np.float32))
        if form == "nt":
            check(lib().tnet_affine_bwd_colsum(dE.ptr, dE.dim, dW.ptr, dW.dim, dY.ptr, dY.stride, dO.ptr, dO.dim,
                                               dP.ptr, dP.stride, S()))
        else:
            check(lib().tnet_affine_bwd_colsum_t(dE.ptr, dE.dim, dT.ptr, dT.dim, dY.ptr, dY.stride, dO.ptr, dO.dim,
                                                 dP.ptr, dP.stride, S()))
        out[form] = (dO.numpy(), dP.numpy())
    (O, P), (O0, P0) = out["t"], out["nt"]
    np.testing.assert_array_equal(O, O0)
    assert np.all(np.abs(P - P0) <= 32 * 1.2e-7 * slab_sums(np.abs(O)) + 1e-7)
    assert np.all(np.abs(P - slab_sums(O)) <= 32 * 1.2e-7 * slab_sums(np.abs(O)) + 1e-7)


@pytest.mark.parametrize("rows,n_in,n_out", [(1024, 2048, 4000), (1024, 2048, 2048)])
def test_bwd_colsum_slabs_t_matches_nt(rows, n_in, n_out):
    """the top layer's backward + the slab sums of its own input error, one launch, from the shadow: Eo bit-identical
    to the NT form, E's slab sums identical (the same blocks), Eo's slab sums within fp32 reordering"""
    E, W = rnd((rows, n_out), 5, 0.01), rnd((n_in, n_out), 6, 0.1)
    Yb = (1 / (1 + np.exp(-rnd((rows, n_in), 7)))).astype(np.float32)
    dE, dW, dY = DeviceArray.from_numpy(E), DeviceArray.from_numpy(W), DeviceArray.from_numpy(Yb)
    dT = transposed(dW)
    slabs = lib().tnet_colsum_slabs(rows)
    out = {}
    for form in ("nt", "t"):
        dO = DeviceArray.from_numpy(np.full((rows, n_in), np.nan, np.float32))
        dP = DeviceArray.from_numpy(np.full((slabs, n_in), np.nan, np.float32))
        dPt = DeviceArray.from_numpy(np.full((slabs, n_out), np.nan, np.float32))
        fn = lib().tnet_affine_bwd_colsum_slabs if form == "nt" else lib().tnet_affine_bwd_colsum_slabs_t
        w = dW if form == "nt" else dT
        st = fn(dE.ptr, dE.dim, w.ptr, w.dim, dY.ptr, dY.stride, dO.ptr, dO.dim, dP.ptr, dP.stride, dPt.ptr,
                dPt.stride, S())
        check(st)
        out[form] = (dO.numpy(), dP.numpy(), dPt.numpy())
    (O, P, Pt), (O0, P0, Pt0) = out["t"], out["nt"]
    np.testing.assert_array_equal(O, O0)
    np.testing.assert_array_equal(Pt, Pt0)
    assert np.all(np.abs(P - P0) <= 32 * 1.2e-7 * slab_sums(np.abs(O)) + 1e-7)


def _register(dW):
    dT = DeviceArray.from_numpy(np.full((dW.cols, dW.rows), np.nan, np.float32))
    check(lib().tnet_weight_shadow(dW.ptr, dW.dim, dT.ptr, dT.stride))
    return dT


def _unregister(dW):
    check(lib().tnet_weight_shadow(dW.ptr, dW.dim, None, 0))


@pytest.mark.parametrize("mmt", [0.0, 0.5])
@pytest.mark.parametrize("rows,n_in,n_out", [(1024, 2048, 2048), (1024, 2048, 4000), (1024, 440, 2048),
                                             (1024, 1024, 135), (1024, 598, 1024), (16, 24, 32)])
def test_update_keeps_shadow(mmt, rows, n_in, n_out):
    """tnet_affine_update_bias with a registered shadow: W identical to the unregistered run, and Wt == W^T exactly
    when tnet_weight_shadow_kept reports it kept (the 16x16 forms; a split-K or 32x32 form reports 0)"""
    X, E = rnd((rows, n_in), 12), rnd((rows, n_out), 13, 0.01)
    W, corr = rnd((n_in, n_out), 14, 0.1), rnd((n_in, n_out), 15, 0.01)
    b, corr_b = rnd(n_out, 18), rnd(n_out, 19, 0.01)
    P = slab_sums(E).astype(np.float32)
    scale, l2 = -0.3 / rows, -1e-4
    res = {}
    for shadow in (True, False):
        dX, dE, dW = DeviceArray.from_numpy(X), DeviceArray.from_numpy(E), DeviceArray.from_numpy(W)
        dP, db = DeviceArray.from_numpy(P), DeviceArray.vector(b)
        dC = DeviceArray.from_numpy(corr) if mmt else None
        dCb = DeviceArray.vector(corr_b) if mmt else None
        dT = _register(dW) if shadow else None
        check(lib().tnet_affine_update_bias(dX.ptr, dX.dim, dE.ptr, dE.dim, dW.ptr, dW.dim, dC.ptr if dC else None,
                                            dC.stride if dC else 0, scale, mmt, l2, dP.ptr, dP.stride, db.ptr,
                                            dCb.ptr if dCb else None, S()))
        synchronize()
        if shadow:
            kept = lib().tnet_weight_shadow_kept(dW.ptr)
            _unregister(dW)
            assert kept in (0, 1)
            if (n_in, n_out) in ((2048, 2048), (2048, 4000), (440, 2048)):
                assert kept == 1, "the step's update forms keep the shadow"
            if kept:
                np.testing.assert_array_equal(dT.numpy(), dW.numpy().T)
        res[shadow] = dW.numpy()
    np.testing.assert_array_equal(res[True], res[False])


@pytest.mark.parametrize("mmt", [0.0, 0.9])
def test_update_bwd_pair_t(mmt):
    """the update + backward pair with the backward from the lower layer's shadow and the update keeping its own:
    W, b, the momentum buffers and Eo identical to the NT pair; the update's shadow == its new W^T"""
    rows, n_in, n_out, n_below = 1024, 2048, 2048, 2048
    X, E = rnd((rows, n_in), 21), rnd((rows, n_out), 22, 0.01)
    W, corr = rnd((n_in, n_out), 23, 0.1), rnd((n_in, n_out), 24, 0.01)
    b, corr_b = rnd(n_out, 25), rnd(n_out, 26, 0.01)
    P = slab_sums(E).astype(np.float32)
    W2, E2 = rnd((n_below, n_in), 27, 0.1), rnd((rows, n_in), 28)
    Yb = (1 / (1 + np.exp(-rnd((rows, n_below), 29)))).astype(np.float32)
    scale, l2 = -0.3 / rows, -1e-4
    slabs = lib().tnet_colsum_slabs(rows)
    res = {}
    for form in ("nt", "t"):
        d = dict(X=DeviceArray.from_numpy(X), E=DeviceArray.from_numpy(E), W=DeviceArray.from_numpy(W),
                 P=DeviceArray.from_numpy(P), b=DeviceArray.vector(b),
                 C=DeviceArray.from_numpy(corr) if mmt else None, Cb=DeviceArray.vector(corr_b) if mmt else None,
                 W2=DeviceArray.from_numpy(W2), E2=DeviceArray.from_numpy(E2), Y=DeviceArray.from_numpy(Yb),
                 O=DeviceArray(rows, n_below), P2=DeviceArray.from_numpy(np.full((slabs, n_below), np.nan, np.float32)))
        C, Cb = d["C"], d["Cb"]
        dT = _register(d["W"]) if form == "t" else None
        w2 = transposed(d["W2"]) if form == "t" else d["W2"]
        args = (d["X"].ptr, d["X"].dim, d["E"].ptr, d["E"].dim, d["W"].ptr, d["W"].dim, C.ptr if C else None,
                C.stride if C else 0, scale, mmt, l2, d["P"].ptr, d["P"].stride, d["b"].ptr, Cb.ptr if Cb else None,
                d["E2"].ptr, d["E2"].dim, w2.ptr, w2.dim, d["Y"].ptr, d["Y"].stride, d["O"].ptr, d["O"].dim,
                d["P2"].ptr, d["P2"].stride, S())
        fn = lib().tnet_affine_update_bwd_pair_t if form == "t" else lib().tnet_affine_update_bwd_pair
        check(fn(*args))
        synchronize()
        if form == "t":
            assert lib().tnet_weight_shadow_kept(d["W"].ptr) == 1
            _unregister(d["W"])
            np.testing.assert_array_equal(dT.numpy(), d["W"].numpy().T)
        res[form] = {k: v.numpy() for k, v in d.items() if v is not None and k in ("W", "b", "C", "Cb", "O", "P2")}
    for k in ("W", "b", "C", "Cb", "O"):
        if k in res["nt"]:
            np.testing.assert_array_equal(res["t"][k], res["nt"][k], err_msg=k)
    O = res["t"]["O"]
    assert np.all(np.abs(res["t"]["P2"] - res["nt"]["P2"]) <= 32 * 1.2e-7 * slab_sums(np.abs(O)) + 1e-7)


@pytest.mark.parametrize("mmt,shadow_top", [(0.0, False), (0.9, False), (0.0, True)])
def test_update_bwd_pair_t_wide(mmt, shadow_top):
    """the top layer's 2048x4000 update (128x256 tiles) paired with the 2048^2 backward below it from that layer's
    shadow (one launch, launch_pair_wide_bwd_t): W, b, the momentum buffers, Eo and the slab sums identical to the
    two separate calls (tnet_affine_update_bias + tnet_affine_bwd_colsum_t); with the top layer's own shadow
    registered its Wt == the new W^T"""
    rows, n_in, n_out, n_below = 1024, 2048, 4000, 2048
    X, E = rnd((rows, n_in), 41), rnd((rows, n_out), 42, 0.01)
    W, corr = rnd((n_in, n_out), 43, 0.1), rnd((n_in, n_out), 44, 0.01)
    b, corr_b = rnd(n_out, 45), rnd(n_out, 46, 0.01)
    P = slab_sums(E).astype(np.float32)
    W2, E2 = rnd((n_below, n_in), 47, 0.1), rnd((rows, n_in), 48)
    Yb = (1 / (1 + np.exp(-rnd((rows, n_below), 49)))).astype(np.float32)
    scale, l2 = -0.3 / rows, -1e-4
    slabs = lib().tnet_colsum_slabs(rows)
    res = {}
    for form in ("pair", "separate"):
        d = dict(X=DeviceArray.from_numpy(X), E=DeviceArray.from_numpy(E), W=DeviceArray.from_numpy(W),
                 P=DeviceArray.from_numpy(P), b=DeviceArray.vector(b),
                 C=DeviceArray.from_numpy(corr) if mmt else None, Cb=DeviceArray.vector(corr_b) if mmt else None,
                 W2=DeviceArray.from_numpy(W2), E2=DeviceArray.from_numpy(E2), Y=DeviceArray.from_numpy(Yb),
                 O=DeviceArray(rows, n_below), P2=DeviceArray.from_numpy(np.full((slabs, n_below), np.nan, np.float32)))
        C, Cb = d["C"], d["Cb"]
        dT = _register(d["W"]) if shadow_top else None
        w2t = transposed(d["W2"])
        upd = (d["X"].ptr, d["X"].dim, d["E"].ptr, d["E"].dim, d["W"].ptr, d["W"].dim, C.ptr if C else None,
               C.stride if C else 0, scale, mmt, l2, d["P"].ptr, d["P"].stride, d["b"].ptr, Cb.ptr if Cb else None)
        bwd = (d["E2"].ptr, d["E2"].dim, w2t.ptr, w2t.dim, d["Y"].ptr, d["Y"].stride, d["O"].ptr, d["O"].dim,
               d["P2"].ptr, d["P2"].stride)
        if form == "pair":
            check(lib().tnet_affine_update_bwd_pair_t(*upd, *bwd, S()))
        else:
            check(lib().tnet_affine_update_bias(*upd, S()))
            check(lib().tnet_affine_bwd_colsum_t(*bwd, S()))
        synchronize()
        if shadow_top:
            if lib().tnet_weight_shadow_kept(d["W"].ptr) == 1:
                np.testing.assert_array_equal(dT.numpy(), d["W"].numpy().T)
            _unregister(d["W"])
        res[form] = {k: v.numpy() for k, v in d.items() if v is not None and k in ("W", "b", "C", "Cb", "O", "P2")}
    for k in res["pair"]:
        np.testing.assert_array_equal(res["pair"][k], res["separate"][k], err_msg=k)


def test_shadow_arguments():
    dW = DeviceArray(64, 32)
    dT = DeviceArray(32, 64)
    assert lib().tnet_weight_shadow_kept(dW.ptr) < 0  # not registered
    check(lib().tnet_weight_shadow(dW.ptr, dW.dim, dT.ptr, dT.stride))
    assert lib().tnet_weight_shadow_kept(dW.ptr) == 0  # no update yet
    assert lib().tnet_weight_shadow(dW.ptr, dW.dim, dT.ptr, 3) != 0  # stride below the row count / unaligned
    _unregister(dW)
    assert lib().tnet_weight_shadow_kept(dW.ptr) < 0


@pytest.mark.parametrize("with_dp", [0, 1])
def test_shadow_across_training_modes(tmp_path, with_dp):
    """ADVICE r5 (medium + low): every writer of W that does not write the transposed shadow -- the generic path's
    one-row update (tnet_affine_update_row), the data-parallel flat apply -- leaves it stale for the next fused
    backward, which must then re-transpose.  The same training sequence (fused, generic 1-row, fused 1-row, fused,
    [DP on a one-rank communicator, fused]) with the shadows on (default) and off (TNET_BWD_SHADOW=0: every backward
    NT from W) ends at the same parameters within the slab-sum reorder band (a stale shadow -- last step's weights
    at lr 2 -- is orders of magnitude outside it).  Tolerance: |p - p0| <= 2e-4 * max|p0| per parameter block."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    got = {}
    for mode in ("2", "0"):
        out = str(tmp_path / f"p{mode}.npz")
        p = subprocess.run([sys.executable, os.path.join(repo, "tests", "shadow_modes_worker.py"), out, str(with_dp)],
                           capture_output=True, text=True, timeout=300, env=dict(os.environ, TNET_BWD_SHADOW=mode))
        assert p.returncode == 0, p.stderr[-3000:]
        got[mode] = dict(np.load(out))
    for k, ref in got["0"].items():
        np.testing.assert_array_less(np.abs(got["2"][k] - ref), 2e-4 * np.abs(ref).max() + 1e-12, err_msg=k)
