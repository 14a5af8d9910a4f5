"""Stream-K over CUs - R workgroups (gemm16_sk_kernel; tnet_gemm_reserve / tnet_gemm_config "+rsv<R>"):
the data-parallel step's GEMM shapes while R CUs are held by RCCL's channel workgroups.  The tiles'
k-tiles are cut into G = CUs - R equal ranges; whole tiles run the plain tile body, pieces at a range's
ends are split-K slices combined in-launch by the tile's last piece.

Tolerances: the same kernel-level bounds as tests/test_gpu_kernels.py (|got - ref| <= 2e-5 (|A||B|) +
1e-7 for GEMM results, slab sums within the fp32 row-sum bound); pieces differ from the whole-tile
body only by their summation order (checked against the fp64 reference, not bitwise); launches are
deterministic (static plan, slices combined in order).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from tnet_amd import DeviceArray, synchronize  # noqa: E402
from tnet_amd._lib import check, lib  # noqa: E402


def S():
    return lib().tnet_stream()


def rnd(shape, seed, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)


def gemm_ref(ta, tb, A, B):
    a = A.astype(np.float64).T if ta == "T" else A.astype(np.float64)
    b = B.astype(np.float64).T if tb == "T" else B.astype(np.float64)
    return a @ b, np.abs(a) @ np.abs(b)


def slab_sums(M, slab=32):
    n = -(-M.shape[0] // slab)
    return np.stack([M[s * slab:(s + 1) * slab].astype(np.float64).sum(0) for s in range(n)])


@pytest.fixture(params=["auto+rsv0", "auto+rsv8", "auto+rsv16", "auto+rsv37", "auto+rsv200", "auto+rsv250"])
def ts_cfg(request):
    check(lib().tnet_gemm_config(request.param.encode()))
    yield request.param
    check(lib().tnet_gemm_config(b"auto+rsv0"))


def _run(cfg, fn):
    check(lib().tnet_gemm_config(cfg.encode()))
    try:
        out = fn()
        synchronize()
        return out
    finally:
        check(lib().tnet_gemm_config(b"auto+rsv0"))


def test_bwd_colsum_stolen(ts_cfg):
    rows, n_in, n_out = 1024, 2048, 2048
    E, W = rnd((rows, n_out), 9), rnd((n_in, n_out), 10, 0.1)
    Yb = (1 / (1 + np.exp(-rnd((rows, n_in), 11)))).astype(np.float32)
    dE, dW, dY = DeviceArray.from_numpy(E), DeviceArray.from_numpy(W), DeviceArray.from_numpy(Yb)
    slabs = lib().tnet_colsum_slabs(rows)
    outs = []
    for _ in range(3):  # consecutive launches: the claim states' double buffer alternates
        dO = DeviceArray(rows, n_in)
        dP = DeviceArray.from_numpy(np.full((slabs, n_in), np.nan, np.float32))
        check(lib().tnet_affine_bwd_colsum(dE.ptr, dE.dim, dW.ptr, dW.dim, dY.ptr, dY.stride, dO.ptr, dO.dim, dP.ptr,
                                           dP.stride, S()))
        outs.append((dO.numpy(), dP.numpy()))
    z, mag = gemm_ref("N", "T", E, W)
    s = Yb * (1 - Yb)
    for got, P in outs:
        assert np.all(np.abs(got - z * s) <= 2e-5 * mag * s + 1e-7)
        assert np.all(np.abs(P - slab_sums(got)) <= 32 * 1.2e-7 * slab_sums(np.abs(got)) + 1e-7)
    np.testing.assert_array_equal(outs[0][0], outs[2][0])  # deterministic launch to launch
    np.testing.assert_array_equal(outs[0][1], outs[2][1])


@pytest.mark.parametrize("with_bias", [True, False])
def test_grad_stolen(ts_cfg, with_bias):
    rows, n_in, n_out = 1024, 2048, 2048
    X, E = rnd((rows, n_in), 12), rnd((rows, n_out), 13, 0.01)
    P = slab_sums(E).astype(np.float32)
    dX, dE, dP = DeviceArray.from_numpy(X), DeviceArray.from_numpy(E), DeviceArray.from_numpy(P)
    g, mag = gemm_ref("T", "N", X, E)
    for _ in range(2):  # deterministic repeats
        dG = DeviceArray(n_in, n_out)
        dgb = DeviceArray.vector(np.full(n_out, np.nan, np.float32))
        if with_bias:
            check(lib().tnet_affine_grad_bias(dX.ptr, dX.dim, dE.ptr, dE.dim, dG.ptr, dG.dim, dP.ptr, dP.stride,
                                              dgb.ptr, S()))
        else:
            check(lib().tnet_affine_grad(dX.ptr, dX.dim, dE.ptr, dE.dim, dG.ptr, dG.dim, S()))
        assert np.all(np.abs(dG.numpy() - g) <= 2e-5 * mag + 1e-7)
        if with_bias:
            np.testing.assert_array_equal(dgb.numpy().ravel(), P.astype(np.float64).sum(0).astype(np.float32))


def test_fwd_stolen(ts_cfg):
    rows, n_in, n_out = 1024, 2048, 2048
    X, W, b = rnd((rows, n_in), 1), rnd((n_in, n_out), 2, 0.05), rnd(n_out, 3)
    dX, dW, db, dY = DeviceArray.from_numpy(X), DeviceArray.from_numpy(W), DeviceArray.vector(b), DeviceArray(rows, n_out)
    check(lib().tnet_affine_fwd(dX.ptr, dX.dim, dW.ptr, dW.dim, db.ptr, dY.ptr, dY.dim, 1, S()))
    z, mag = gemm_ref("N", "N", X, W)
    y = 1 / (1 + np.exp(-(z + b)))
    s = y * (1 - y)
    assert np.all(np.abs(dY.numpy() - y) <= 2e-5 * mag * s + 1e-6)


def test_reserve_api():
    assert lib().tnet_gemm_reserve(-1) != 0
    check(lib().tnet_gemm_reserve(8))
    check(lib().tnet_gemm_reserve(0))
    assert lib().tnet_gemm_config(b"auto+rsvx") != 0


@pytest.fixture
def split2():
    check(lib().tnet_gemm_config(b"auto+s21"))  # opt-in (measured slower than 64x64 tiles over the whole K)
    yield
    check(lib().tnet_gemm_config(b"auto+s20"))


@pytest.mark.parametrize("kind", ["updb", "upd", "gradb"])
def test_update_split2_first_layer(split2, kind):
    """gemm16_split2_kernel (the first layer's 440 x 2048 update over K = 1024: 112 tiles of 64x128, each
    cut into two k-halves combined by the stream-K fixup before the fused SGD / bias epilogue; the last
    tile-row is partial, rows 440..447 masked): against the fp64 update, bias from the slab sums,
    deterministic launch to launch."""
    rows, n_in, n_out, scale = 1024, 440, 2048, -0.5
    X, E = rnd((rows, n_in), 21), rnd((rows, n_out), 22, 0.01)
    W0 = rnd((n_in, n_out), 23, 0.05)
    b0 = rnd(n_out, 24, 0.1)
    P = slab_sums(E).astype(np.float32)
    g, mag = gemm_ref("T", "N", X, E)
    outs = []
    for _ in range(2):
        dX, dE, dP = DeviceArray.from_numpy(X), DeviceArray.from_numpy(E), DeviceArray.from_numpy(P)
        dW, db = DeviceArray.from_numpy(W0), DeviceArray.vector(b0)
        if kind == "updb":
            check(lib().tnet_affine_update_bias(dX.ptr, dX.dim, dE.ptr, dE.dim, dW.ptr, dW.dim, None, 0,
                                                ctypes.c_float(scale), ctypes.c_float(0.0), ctypes.c_float(0.0),
                                                dP.ptr, dP.stride, db.ptr, None, S()))
        elif kind == "upd":
            check(lib().tnet_affine_update(dX.ptr, dX.dim, dE.ptr, dE.dim, dW.ptr, dW.dim, None, 0,
                                           ctypes.c_float(scale), ctypes.c_float(0.0), ctypes.c_float(0.0), S()))
        else:
            dW = DeviceArray(n_in, n_out)
            db = DeviceArray.vector(np.full(n_out, np.nan, np.float32))
            check(lib().tnet_affine_grad_bias(dX.ptr, dX.dim, dE.ptr, dE.dim, dW.ptr, dW.dim, dP.ptr, dP.stride,
                                              db.ptr, S()))
        synchronize()
        outs.append((dW.numpy(), db.numpy().ravel()))
    Wg, bg = outs[0]
    if kind == "gradb":
        assert np.all(np.abs(Wg - g) <= 2e-5 * mag + 1e-7)
        np.testing.assert_array_equal(bg, P.astype(np.float64).sum(0).astype(np.float32))
    else:
        want = W0.astype(np.float64) + scale * g
        assert np.all(np.abs(Wg - want) <= abs(scale) * 2e-5 * mag + 2 * np.spacing(np.abs(want)) + 1e-7)
        if kind == "updb":
            bw = (b0 + np.float32(scale) * P.astype(np.float64).sum(0).astype(np.float32)).astype(np.float32)
            np.testing.assert_allclose(bg, bw, rtol=0, atol=2 * np.spacing(np.abs(bw)).max())
        else:
            np.testing.assert_array_equal(bg, b0)
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
