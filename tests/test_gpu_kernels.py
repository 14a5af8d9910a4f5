"""Kernel-level parity of the gfx950 HIP kernels (through the C ABI) against the oracle.

Floating-point tolerances (fp32 in / fp32 accumulate vs an fp64-accumulated checker):
  GEMM-shaped results: |got - ref| <= 2e-5 * (|A||B|)_ij + 1e-6  (k-ordered f32 FMA chain, K <= 4096)
  element-wise maps:   rtol 2e-6 (expf/logf vs libm double)
  reductions:          rtol 1e-5
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle as orc  # noqa: E402
from tnet_amd import DeviceArray, _lib, synchronize  # noqa: E402
from tnet_amd._lib import MatrixDim, check, lib  # noqa: E402


TNET_ERR_ARG, TNET_ERR_UNSUPPORTED = -1, -4  # include/tnet_kernels.h


def S():
    """the library stream: kernels and the DeviceArray copies must be stream-ordered"""
    return lib().tnet_stream()


def rnd(shape, seed, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)


def gemm_ref(ta, tb, A, B):
    a = A.astype(np.float64).T if ta == "T" else A.astype(np.float64)
    b = B.astype(np.float64).T if tb == "T" else B.astype(np.float64)
    return a @ b, np.abs(a) @ np.abs(b)


GEMM_CFGS = ["auto", "g64x64k32s4w4", "m64x64k32s4w41", "m128x128k64s2", "m64x128k64s2", "m128x256k32s3",
             "m64x64k64s2", "m64x64k32s4", "m32x64k64s2",
             # the direct form (fragments loaded into a register ring, no LDS ring; exact shapes only,
             # the ring form otherwise)
             "m64x128a4", "m64x128a8", "m128x128a4", "m128x256a2", "m64x64a4",
             # ... with the k-contiguous operands' loads coalesced and the fragments moved by ds_bpermute
             "m64x128c8",
             # split-K (K cut into slices + an in-order combine with the epilogue); counts that do not
             # divide K fall back to fewer slices
             "auto+sk4", "m64x64k32s4w41+sk8", "m32x64k64s2+sk2", "m64x128k64s2+sk3", "m64x64k32s4w41+sk2",
             "m64x64k32s4w41+sk4", "m32x64k64s2+sk8", "m128x128k64s2+sk2"]


@pytest.fixture(params=GEMM_CFGS)
def gemm_cfg(request):
    check(lib().tnet_gemm_config(request.param.encode()))
    yield request.param
    check(lib().tnet_gemm_config(b"auto"))


GEMM_SHAPES = [(1, 1, 1), (7, 5, 3), (33, 65, 31), (64, 64, 32), (130, 70, 598), (200, 135, 1024),
               (256, 384, 440), (1024, 2048, 2048), (1024, 4000, 2048), (2048, 2048, 1024), (440, 2048, 1024)]


@pytest.mark.parametrize("ta,tb", [("N", "N"), ("N", "T"), ("T", "N"), ("T", "T")])
@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
def test_sgemm(ta, tb, M, N, K, gemm_cfg):
    A = rnd((K, M) if ta == "T" else (M, K), 1)
    B = rnd((N, K) if tb == "T" else (K, N), 2)
    C0 = rnd((M, N), 3)
    alpha, beta = 0.75, 0.5
    dA, dB, dC = DeviceArray.from_numpy(A), DeviceArray.from_numpy(B), DeviceArray.from_numpy(C0)
    check(lib().tnet_sgemm(ta.encode(), tb.encode(), M, N, K, alpha, dA.ptr, dA.stride, dB.ptr, dB.stride, beta,
                           dC.ptr, dC.stride, S()), "sgemm")
    got = dC.numpy()
    ref, mag = gemm_ref(ta, tb, A, B)
    ref = alpha * ref + beta * C0
    err = np.abs(got - ref)
    assert np.all(err <= 2e-5 * (alpha * mag + np.abs(beta * C0)) + 1e-6), err.max()


def test_sgemm_beta_zero_ignores_garbage():
    M, N, K = 70, 90, 50
    A, B = rnd((M, K), 4), rnd((K, N), 5)
    dA, dB = DeviceArray.from_numpy(A), DeviceArray.from_numpy(B)
    dC = DeviceArray.from_numpy(np.full((M, N), np.nan, np.float32))
    check(lib().tnet_sgemm(b"N", b"N", M, N, K, 1.0, dA.ptr, dA.stride, dB.ptr, dB.stride, 0.0, dC.ptr, dC.stride,
                           S()))
    assert np.isfinite(dC.numpy()).all()


def test_sgemm_rejects_misaligned_stride():
    d = DeviceArray(8, 8)
    st = lib().tnet_sgemm(b"N", b"N", 8, 8, 8, 1.0, d.ptr, 6, d.ptr, 8, 0.0, d.ptr, 8, S())
    assert st == -1


@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("rows,n_in,n_out", [(16, 24, 32), (1024, 440, 2048), (960, 598, 1024), (33, 1024, 135)])
def test_affine_fwd(act, rows, n_in, n_out, gemm_cfg):
    X, W, b = rnd((rows, n_in), 6), rnd((n_in, n_out), 7, 0.1), rnd(n_out, 8)
    dX, dW, dY = DeviceArray.from_numpy(X), DeviceArray.from_numpy(W), DeviceArray(rows, n_out)
    db = DeviceArray.vector(b)
    check(lib().tnet_affine_fwd(dX.ptr, dX.dim, dW.ptr, dW.dim, db.ptr, dY.ptr, dY.dim, act, S()))
    z, mag = gemm_ref("N", "N", X, W)
    z = z + b
    got = dY.numpy()
    if act:
        ref = 1.0 / (1.0 + np.exp(-z))
        assert np.all(np.abs(got - ref) <= 2e-5 * mag * ref * (1 - ref) + 2e-6)
    else:
        assert np.all(np.abs(got - z) <= 2e-5 * mag + 1e-6)


@pytest.mark.parametrize("rows,n_in,n_out", [(16, 32, 10), (45, 37, 50), (1024, 2048, 2048), (1024, 2048, 4000)])
def test_affine_bwd_dsig(rows, n_in, n_out, gemm_cfg):
    E, W = rnd((rows, n_out), 9), rnd((n_in, n_out), 10, 0.1)
    Yb = 1 / (1 + np.exp(-rnd((rows, n_in), 11)))
    dE, dW, dY, dO = (DeviceArray.from_numpy(E), DeviceArray.from_numpy(W), DeviceArray.from_numpy(Yb),
                      DeviceArray(rows, n_in))
    check(lib().tnet_affine_bwd(dE.ptr, dE.dim, dW.ptr, dW.dim, dY.ptr, dY.stride, dO.ptr, dO.dim, 1, S()))
    z, mag = gemm_ref("N", "T", E, W)
    s = Yb * (1 - Yb)
    assert np.all(np.abs(dO.numpy() - z * s) <= 2e-5 * mag * s + 1e-7)


@pytest.mark.parametrize("mmt", [0.0, 0.5])
@pytest.mark.parametrize("rows,n_in,n_out", [(16, 24, 32), (1024, 2048, 2048), (1024, 440, 2048), (960, 1024, 135)])
def test_affine_update(mmt, rows, n_in, n_out, gemm_cfg):
    X, E = rnd((rows, n_in), 12), rnd((rows, n_out), 13, 0.01)
    W, corr = rnd((n_in, n_out), 14, 0.1), rnd((n_in, n_out), 15, 0.01)
    scale, l2 = -0.3 / rows, -1e-4
    dX, dE, dW = DeviceArray.from_numpy(X), DeviceArray.from_numpy(E), DeviceArray.from_numpy(W)
    dC = DeviceArray.from_numpy(corr) if mmt else None
    check(lib().tnet_affine_update(dX.ptr, dX.dim, dE.ptr, dE.dim, dW.ptr, dW.dim, dC.ptr if dC else None,
                                   dC.stride if dC else 0, scale, mmt, l2, S()))
    g, mag = gemm_ref("T", "N", X, E)
    c = g + mmt * corr
    w = W + scale * c
    w = w + l2 * w
    tol = 2e-5 * abs(scale) * mag + 2e-7 * np.abs(W) + 1e-7
    assert np.all(np.abs(dW.numpy() - w) <= tol)
    if mmt:
        assert np.all(np.abs(dC.numpy() - c) <= 2e-5 * mag + 1e-6)


@pytest.mark.parametrize("sides", [[(1024, 135), (598, 1024)], [(2048, 2048), (440, 2048)]])
def test_affine_grad_pair_gather(sides):
    """tnet_affine_grad_bias_gather with two gradients (MLP3's last two layers in a data-parallel step) and the next
    bunch's gather in ONE launch: each G / bias gradient against the fp64 XᵀE and the slab sums (the pair runs the
    64x64 tiles unsplit, so the standalone call -- split-K for 1024x135 -- is not bit-identical), the gathered rows
    and class ids exact; TNET_ERR_UNSUPPORTED where the two grids do not fit one round (dnn4's 2048² + 440x2048)"""
    rows, gcols = 1024, 598
    Xc = rnd((3000, gcols), 600)
    labc = (np.arange(3000, dtype=np.int32) * 7) % 4000
    perm = np.random.default_rng(601).permutation(3000).astype(np.int32)[:1024]
    host, dev, args = [], [], []
    for k, (n_in, n_out) in enumerate(sides):
        X, E = rnd((rows, n_in), 610 + k), rnd((rows, n_out), 620 + k, 0.01)
        host.append((X, E))
        d = dict(X=DeviceArray.from_numpy(X), E=DeviceArray.from_numpy(E), P=DeviceArray.from_numpy(slab_sums(E).astype(np.float32)),
                 G=DeviceArray.from_numpy(np.full((n_in, n_out), np.nan, np.float32)),
                 gb=DeviceArray.vector(np.full(n_out, np.nan, np.float32)))
        dev.append(d)
        args.append([d["X"].ptr, d["X"].dim, d["E"].ptr, d["E"].dim, d["G"].ptr, d["G"].dim, d["P"].ptr, d["P"].stride,
                     d["gb"].ptr])
    dXc, dLc, dPerm = DeviceArray.from_numpy(Xc), DeviceArray.vector(labc), DeviceArray.vector(perm)
    dY = DeviceArray.from_numpy(np.full((1024, gcols), np.nan, np.float32))
    dLo = DeviceArray.vector(np.full(1024, -7, np.int32))
    st = lib().tnet_affine_grad_bias_gather(*args[0], *args[1], dY.ptr, dXc.ptr, dLo.ptr, dLc.ptr, dPerm.ptr, dY.dim,
                                            dXc.dim, S())
    if sides[0] == (2048, 2048):
        assert st == TNET_ERR_UNSUPPORTED
        return
    check(st)
    for (X, E), d in zip(host, dev):
        np.testing.assert_allclose(d["G"].numpy(), X.astype(np.float64).T @ E.astype(np.float64), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(d["gb"].numpy().ravel(), E.astype(np.float64).sum(0), rtol=1e-4, atol=1e-5)
    np.testing.assert_array_equal(dY.numpy(), Xc[perm])
    np.testing.assert_array_equal(dLo.numpy()[:, 0], labc[perm])


@pytest.mark.parametrize("direct,ring", [("m64x128a4", "m64x128k64s2"), ("m64x128a8", "m64x128k64s2"),
                                         ("m128x128a4", "m128x128k64s2"), ("m128x256a2", "m128x256k32s3"),
                                         ("m64x128c8", "m64x128k64s2"), ("m64x64a4", "m64x64k64s2")])
@pytest.mark.parametrize("kind,rows,n_in,n_out", [("fwd", 1024, 2048, 2048), ("bwd", 1024, 2048, 2048),
                                                  ("upd", 1024, 2048, 2048), ("upd", 1024, 2048, 4096),
                                                  ("bwd", 1024, 2048, 4000), ("bwd", 1000, 1000, 4000),
                                                  ("fwd", 1000, 440, 2048)])
def test_direct_form_bit_identical_to_ring(direct, ring, kind, rows, n_in, n_out):
    """the GEMM's direct form (each wave loads its MFMA fragments from global memory into a register ring) runs
    the ring form's MFMA sequence on the same operand values in the same order: the outputs bit for bit"""
    X, E = rnd((rows, n_in), 60), rnd((rows, n_out), 61, 0.01)
    W, b = rnd((n_in, n_out), 62, 0.1), rnd(n_out, 63)
    Yb = 1 / (1 + np.exp(-rnd((rows, n_in), 64)))
    out = []
    for cfg in (direct, ring):
        check(lib().tnet_gemm_config(cfg.encode()))
        try:
            dX, dE, dW, db, dY = (DeviceArray.from_numpy(X), DeviceArray.from_numpy(E), DeviceArray.from_numpy(W),
                                  DeviceArray.vector(b), DeviceArray.from_numpy(Yb))
            if kind == "fwd":
                dO = DeviceArray(rows, n_out)
                check(lib().tnet_affine_fwd(dX.ptr, dX.dim, dW.ptr, dW.dim, db.ptr, dO.ptr, dO.dim, 1, S()))
                out.append(dO.numpy())
            elif kind == "bwd":
                dO = DeviceArray(rows, n_in)
                check(lib().tnet_affine_bwd(dE.ptr, dE.dim, dW.ptr, dW.dim, dY.ptr, dY.stride, dO.ptr, dO.dim, 1, S()))
                out.append(dO.numpy())
            else:
                check(lib().tnet_affine_update(dX.ptr, dX.dim, dE.ptr, dE.dim, dW.ptr, dW.dim, None, 0, -0.3 / rows, 0.0,
                                               -1e-4, S()))
                out.append(dW.numpy())
        finally:
            check(lib().tnet_gemm_config(b"auto"))
    np.testing.assert_array_equal(out[0], out[1])


def slab_sums(M, slab=32):
    """column sums of M per 32-row slab (fp64)"""
    n = -(-M.shape[0] // slab)
    return np.stack([M[s * slab:(s + 1) * slab].astype(np.float64).sum(0) for s in range(n)])


@pytest.fixture(params=["auto", "m64x128k64s2", "m64x64k32s4", "m64x64k64s2"])
def colsum_cfg(request):
    """the configurations the column-sum bwd accepts (32-row wave tiles)"""
    check(lib().tnet_gemm_config(request.param.encode()))
    yield request.param
    check(lib().tnet_gemm_config(b"auto"))


@pytest.mark.parametrize("rows,n_in,n_out", [(16, 32, 10), (33, 64, 40), (45, 37, 50), (1024, 2048, 2048),
                                             (1000, 440, 2048), (1024, 2048, 4000), (1024, 1024, 135)])
def test_affine_bwd_colsum(rows, n_in, n_out, colsum_cfg):
    """bwd + diff-sigmoid with the bias gradient of the layer below as 32-row slab column sums (every
    configuration with 32-row wave tiles)"""
    E, W = rnd((rows, n_out), 9), rnd((n_in, n_out), 10, 0.1)
    Yb = 1 / (1 + np.exp(-rnd((rows, n_in), 11)))
    dE, dW, dY, dO = (DeviceArray.from_numpy(E), DeviceArray.from_numpy(W), DeviceArray.from_numpy(Yb),
                      DeviceArray(rows, n_in))
    slabs = lib().tnet_colsum_slabs(rows)
    assert slabs == -(-rows // 32)
    dP = DeviceArray.from_numpy(np.full((slabs, n_in), np.nan, np.float32))
    check(lib().tnet_affine_bwd_colsum(dE.ptr, dE.dim, dW.ptr, dW.dim, dY.ptr, dY.stride, dO.ptr, dO.dim, dP.ptr,
                                       dP.stride, S()))
    z, mag = gemm_ref("N", "T", E, W)
    s = Yb * (1 - Yb)
    got = dO.numpy()
    assert np.all(np.abs(got - z * s) <= 2e-5 * mag * s + 1e-7)
    # slab sums: each is the fp32 sum (in row order) of the kernel's own outputs
    P = dP.numpy()
    ref = slab_sums(z * s)
    tol = slab_sums(2e-5 * mag * s + 1e-7) + 32 * 6e-8 * slab_sums(np.abs(got))
    assert np.all(np.abs(P - ref) <= tol)
    assert np.all(np.abs(P - slab_sums(got)) <= 32 * 1.2e-7 * slab_sums(np.abs(got)) + 1e-7)


@pytest.mark.parametrize("mmt", [0.0, 0.5])
@pytest.mark.parametrize("rows,n_in,n_out", [(16, 24, 32), (1024, 2048, 2048), (1024, 440, 2048), (960, 1024, 135),
                                             (1024, 1024, 135), (1024, 598, 1024), (1024, 2048, 4000)])
def test_affine_update_bias(mmt, rows, n_in, n_out, gemm_cfg):
    """weight SGD + bias SGD (bias gradient from slab sums) in one launch"""
    X, E = rnd((rows, n_in), 12), rnd((rows, n_out), 13, 0.01)
    W, corr = rnd((n_in, n_out), 14, 0.1), rnd((n_in, n_out), 15, 0.01)
    b, corr_b = rnd(n_out, 18), rnd(n_out, 19, 0.01)
    P = slab_sums(E).astype(np.float32)
    scale, l2 = -0.3 / rows, -1e-4
    dX, dE, dW = DeviceArray.from_numpy(X), DeviceArray.from_numpy(E), DeviceArray.from_numpy(W)
    dP, db = DeviceArray.from_numpy(P), DeviceArray.vector(b)
    dC = DeviceArray.from_numpy(corr) if mmt else None
    dCb = DeviceArray.vector(corr_b) if mmt else None
    check(lib().tnet_affine_update_bias(dX.ptr, dX.dim, dE.ptr, dE.dim, dW.ptr, dW.dim, dC.ptr if dC else None,
                                        dC.stride if dC else 0, scale, mmt, l2, dP.ptr, dP.stride, db.ptr,
                                        dCb.ptr if dCb else None, S()))
    g, mag = gemm_ref("T", "N", X, E)
    c = g + mmt * corr
    w = W + scale * c
    w = w + l2 * w
    tol = 2e-5 * abs(scale) * mag + 2e-7 * np.abs(W) + 1e-7
    assert np.all(np.abs(dW.numpy() - w) <= tol)
    if mmt:
        assert np.all(np.abs(dC.numpy() - c) <= 2e-5 * mag + 1e-6)
    gb = P.astype(np.float64).sum(0).astype(np.float32).astype(np.float64)
    cb = gb + mmt * corr_b
    np.testing.assert_allclose(db.numpy().ravel(), b + scale * cb, rtol=1e-6, atol=1e-7)
    if mmt:
        np.testing.assert_allclose(dCb.numpy().ravel(), cb, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("mmt", [0.0, 0.5])
@pytest.mark.parametrize("rows,n_in,n_out,n_below", [(1024, 2048, 2048, 2048), (1024, 2048, 4000, 2048),
                                                     (2048, 2048, 2048, 2048), (1024, 1024, 2048, 1024)])
def test_affine_update_bwd_pair(mmt, rows, n_in, n_out, n_below):
    """tnet_affine_update_bwd_pair (layer l's fused update + layer l-1's backward GEMM in one launch)
    gives exactly what the two calls give (same tile bodies: bit-identical), or declines with
    TNET_ERR_UNSUPPORTED where the pair kernel does not take the shapes"""
    X, E = rnd((rows, n_in), 21), rnd((rows, n_out), 22, 0.01)
    W, corr = rnd((n_in, n_out), 23, 0.1), rnd((n_in, n_out), 24, 0.01)
    b, corr_b = rnd(n_out, 25), rnd(n_out, 26, 0.01)
    P = slab_sums(E).astype(np.float32)
    # layer below: W2 [n_below x n_in], E2 = the error at its output [rows x n_in], Yb its input's y
    W2, E2 = rnd((n_below, n_in), 27, 0.1), rnd((rows, n_in), 28)
    Yb = (1 / (1 + np.exp(-rnd((rows, n_below), 29)))).astype(np.float32)
    scale, l2 = -0.3 / rows, -1e-4
    slabs = lib().tnet_colsum_slabs(rows)

    def run(pair):
        d = dict(X=DeviceArray.from_numpy(X), E=DeviceArray.from_numpy(E), W=DeviceArray.from_numpy(W),
                 P=DeviceArray.from_numpy(P), b=DeviceArray.vector(b),
                 C=DeviceArray.from_numpy(corr) if mmt else None, Cb=DeviceArray.vector(corr_b) if mmt else None,
                 W2=DeviceArray.from_numpy(W2), E2=DeviceArray.from_numpy(E2), Y=DeviceArray.from_numpy(Yb),
                 O=DeviceArray(rows, n_below), P2=DeviceArray.from_numpy(np.full((slabs, n_below), np.nan, np.float32)))
        C, Cb = d["C"], d["Cb"]
        upd = (d["X"].ptr, d["X"].dim, d["E"].ptr, d["E"].dim, d["W"].ptr, d["W"].dim, C.ptr if C else None,
               C.stride if C else 0, scale, mmt, l2, d["P"].ptr, d["P"].stride, d["b"].ptr, Cb.ptr if Cb else None)
        bwd = (d["E2"].ptr, d["E2"].dim, d["W2"].ptr, d["W2"].dim, d["Y"].ptr, d["Y"].stride, d["O"].ptr, d["O"].dim,
               d["P2"].ptr, d["P2"].stride)
        if pair:
            st = lib().tnet_affine_update_bwd_pair(*upd, *bwd, S())
            if st == TNET_ERR_UNSUPPORTED:
                return None
            check(st)
        else:
            check(lib().tnet_affine_update_bias(*upd, S()))
            check(lib().tnet_affine_bwd_colsum(*bwd, S()))
        synchronize()
        return {k: v.numpy() for k, v in d.items() if v is not None and k in ("W", "b", "C", "Cb", "O", "P2")}

    got, ref = run(True), run(False)
    if (n_in, n_out, n_below) == (2048, 2048, 2048):
        assert got is not None, "the step's 2048-wide layers must run as one launch"
    if n_out == 4000:  # the planner gives that update 128x256 tiles: not the pair kernel's
        assert got is None
    if got is None:
        return
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


@pytest.mark.parametrize("rows,n_in,n_out,n_below", [(1024, 2048, 2048, 2048), (1024, 2048, 4000, 2048),
                                                     (1024, 1024, 2048, 1024)])
def test_affine_grad_bwd_pair(rows, n_in, n_out, n_below):
    """tnet_affine_grad_bwd_pair (the data-parallel step's gradient of layer l + layer l-1's backward GEMM in one
    launch) gives exactly what tnet_affine_grad_bias + tnet_affine_bwd_colsum give, or declines with
    TNET_ERR_UNSUPPORTED where the pair kernel does not take the shapes, and while CUs are reserved for RCCL"""
    X, E = rnd((rows, n_in), 31), rnd((rows, n_out), 32, 0.01)
    P = slab_sums(E).astype(np.float32)
    W2, E2 = rnd((n_below, n_in), 37, 0.1), rnd((rows, n_in), 38)
    Yb = (1 / (1 + np.exp(-rnd((rows, n_below), 39)))).astype(np.float32)
    slabs = lib().tnet_colsum_slabs(rows)

    def run(pair, reserve=0):
        d = dict(X=DeviceArray.from_numpy(X), E=DeviceArray.from_numpy(E), P=DeviceArray.from_numpy(P),
                 G=DeviceArray.from_numpy(np.full((n_in, n_out), np.nan, np.float32)),
                 gb=DeviceArray.vector(np.full(n_out, np.nan, np.float32)),
                 W2=DeviceArray.from_numpy(W2), E2=DeviceArray.from_numpy(E2), Y=DeviceArray.from_numpy(Yb),
                 O=DeviceArray(rows, n_below), P2=DeviceArray.from_numpy(np.full((slabs, n_below), np.nan, np.float32)))
        grad = (d["X"].ptr, d["X"].dim, d["E"].ptr, d["E"].dim, d["G"].ptr, d["G"].dim, d["P"].ptr, d["P"].stride,
                d["gb"].ptr)
        bwd = (d["E2"].ptr, d["E2"].dim, d["W2"].ptr, d["W2"].dim, d["Y"].ptr, d["Y"].stride, d["O"].ptr, d["O"].dim,
               d["P2"].ptr, d["P2"].stride)
        if pair:
            check(lib().tnet_gemm_reserve(reserve))
            try:
                st = lib().tnet_affine_grad_bwd_pair(*grad, *bwd, S())
            finally:
                check(lib().tnet_gemm_reserve(0))
            if st == TNET_ERR_UNSUPPORTED:
                return None
            check(st)
        else:
            check(lib().tnet_affine_grad_bias(*grad, S()))
            check(lib().tnet_affine_bwd_colsum(*bwd, S()))
        synchronize()
        return {k: v.numpy() for k, v in d.items() if k in ("G", "gb", "O", "P2")}

    got, ref = run(True), run(False)
    if (n_in, n_out, n_below) == (2048, 2048, 2048):
        assert got is not None, "the step's 2048-wide layers must run as one launch"
        assert run(True, reserve=16) is None, "no pair while CUs are reserved for RCCL"
    if got is None:
        return
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    np.testing.assert_allclose(ref["G"], X.astype(np.float64).T @ E.astype(np.float64), rtol=1e-4, atol=1e-5)


def test_affine_update_bwd_pair_rejects_shared_weights():
    X, E = rnd((64, 128), 1), rnd((64, 128), 2)
    dX, dE, dW, dP, db = (DeviceArray.from_numpy(X), DeviceArray.from_numpy(E), DeviceArray(128, 128),
                          DeviceArray(2, 128), DeviceArray.vector(np.zeros(128, np.float32)))
    dY, dO, dP2 = DeviceArray(64, 128), DeviceArray(64, 128), DeviceArray(2, 128)
    st = lib().tnet_affine_update_bwd_pair(dX.ptr, dX.dim, dE.ptr, dE.dim, dW.ptr, dW.dim, None, 0, -0.1, 0.0, 0.0,
                                           dP.ptr, dP.stride, db.ptr, None, dE.ptr, dE.dim, dW.ptr, dW.dim, dY.ptr,
                                           dY.stride, dO.ptr, dO.dim, dP2.ptr, dP2.stride, S())
    assert st == TNET_ERR_ARG


@pytest.mark.parametrize("rows,n_in,n_out", [(16, 24, 32), (1024, 2048, 2048), (1024, 440, 2048), (1000, 2048, 4000),
                                             (1024, 1024, 135)])
def test_affine_grad_bias(rows, n_in, n_out, gemm_cfg):
    """data-parallel gradient: G = X^T E and gradB = colsum(E) from slab sums, one launch"""
    X, E = rnd((rows, n_in), 12), rnd((rows, n_out), 13, 0.01)
    P = slab_sums(E).astype(np.float32)
    dX, dE, dG = DeviceArray.from_numpy(X), DeviceArray.from_numpy(E), DeviceArray(n_in, n_out)
    dP, dgb = DeviceArray.from_numpy(P), DeviceArray.vector(np.full(n_out, np.nan, np.float32))
    check(lib().tnet_affine_grad_bias(dX.ptr, dX.dim, dE.ptr, dE.dim, dG.ptr, dG.dim, dP.ptr, dP.stride, dgb.ptr, S()))
    g, mag = gemm_ref("T", "N", X, E)
    assert np.all(np.abs(dG.numpy() - g) <= 2e-5 * mag + 1e-7)
    np.testing.assert_array_equal(dgb.numpy().ravel(), P.astype(np.float64).sum(0).astype(np.float32))


@pytest.fixture(params=["auto", "auto+sk4", "m64x128k64s2", "m32x64k64s2+sk2", "g64x64k32s4w4"])
def top_cfg(request):
    """GEMM configurations of the top layer ("auto": the K-slice kernel of top_rows.hip for the shapes it takes,
    the general split-K tiles for the rest)"""
    check(lib().tnet_gemm_config(request.param.encode()))
    yield request.param
    check(lib().tnet_gemm_config(b"auto"))


@pytest.mark.parametrize("keep_y", [False, True])
@pytest.mark.parametrize("rows,n_in,n_out", [(1024, 1024, 135), (37, 20, 7), (1000, 598, 256), (64, 1024, 128),
                                             (300, 2048, 200), (1, 5, 1), (1000, 512, 135), (80, 768, 144),
                                             (1009, 1024, 17)])
def test_affine_softmax_xent(rows, n_in, n_out, keep_y, top_cfg):
    """the fused top layer (slices + bias + softmax + xent + error + slab sums) gives the logits, the
    softmax output and the error of tnet_affine_fwd + tnet_softmax_xent bit for bit, their statistics,
    and slab sums of its own error"""
    X, W, b = rnd((rows, n_in), 60), rnd((n_in, n_out), 61, 0.1), rnd(n_out, 62)
    lab = np.random.default_rng(63).integers(0, n_out, size=rows).astype(np.int32)
    lab[::7] = -1
    lab[3::11] = n_out - 1
    dX, dW, db, dL = (DeviceArray.from_numpy(X), DeviceArray.from_numpy(W), DeviceArray.vector(b),
                      DeviceArray.vector(lab))
    slabs = lib().tnet_colsum_slabs(rows)
    res = []
    for fused in (True, False):
        dZ, dE = DeviceArray(rows, n_out), DeviceArray(rows, n_out)
        dY = DeviceArray(rows, n_out) if keep_y else None
        stats = DeviceArray(1, 1024, np.float64, stride=1024)
        dP = DeviceArray.from_numpy(np.full((slabs, n_out), np.nan, np.float32))
        yp, ys = (dY.ptr, dY.stride) if keep_y else (None, 0)
        if fused:
            check(lib().tnet_affine_softmax_xent(dX.ptr, dX.dim, dW.ptr, dW.dim, db.ptr, dL.ptr, dZ.ptr, dZ.stride,
                                                 yp, ys, dE.ptr, dE.stride, stats.ptr, dP.ptr, dP.stride, S()))
        else:
            check(lib().tnet_affine_fwd(dX.ptr, dX.dim, dW.ptr, dW.dim, db.ptr, dZ.ptr, dZ.dim, 0, S()))
            check(lib().tnet_softmax_xent(dZ.ptr, dZ.dim, dL.ptr, yp, ys, dE.ptr, dE.stride, stats.ptr, S()))
        s = stats.numpy()[0]
        res.append((dZ.numpy(), dY.numpy() if keep_y else None, dE.numpy(), s[0::2].sum(), s[1::2].sum(),
                    dP.numpy()))
    (Z, Y, E, xe, cor, P), (Z0, Y0, E0, xe0, cor0, _) = res
    if top_cfg != "g64x64k32s4w4":  # that 32x32x2 kernel has no slice form: the fused path takes 16x16x4 tiles
        np.testing.assert_array_equal(Z, Z0)
        np.testing.assert_array_equal(E, E0)
        if keep_y:
            np.testing.assert_array_equal(Y, Y0)
        np.testing.assert_allclose(xe, xe0, rtol=1e-12, atol=1e-12)
        assert cor == cor0
    # and the objective itself against the oracle
    z, mag = gemm_ref("N", "N", X, W)
    assert np.all(np.abs(Z - (z + b)) <= 2e-5 * mag + 1e-6)
    Yref = orc.softmax(Z)
    Eref, xent, correct = orc.xent_eval(Yref, lab)
    np.testing.assert_allclose(E, Eref, rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(xe, xent, rtol=1e-5, atol=1e-5)
    assert int(round(cor)) == correct
    # slab sums: fp32 in row order over the slab's rows of E
    ref = slab_sums(E)
    assert np.all(np.abs(P - ref) <= 32 * 1.2e-7 * slab_sums(np.abs(E)) + 1e-7)


def test_affine_softmax_xent_limits():
    """more than TNET_AFFINE_SOFTMAX_MAX_N classes: unsupported (the caller takes the three calls)"""
    X, W, b = rnd((8, 4), 64), rnd((4, 257), 65), rnd(257, 66)
    dX, dW, db = DeviceArray.from_numpy(X), DeviceArray.from_numpy(W), DeviceArray.vector(b)
    dL, dE = DeviceArray.vector(np.zeros(8, np.int32)), DeviceArray(8, 257)
    assert lib().tnet_affine_softmax_xent(dX.ptr, dX.dim, dW.ptr, dW.dim, db.ptr, dL.ptr, None, 0, None, 0, dE.ptr,
                                          dE.stride, None, None, 0, S()) == -4
    assert lib().tnet_affine_softmax_xent(dX.ptr, dX.dim, dW.ptr, dW.dim, None, dL.ptr, None, 0, None, 0, dE.ptr,
                                          dE.stride, None, None, 0, S()) == -1


@pytest.mark.parametrize("mmt", [0.0, 0.9])
@pytest.mark.parametrize("n_in,n_out", [(1, 1), (512, 135), (440, 2048), (37, 4001)])
def test_affine_update_row(mmt, n_in, n_out):
    """one-frame weight + bias SGD in one launch (TRecurrentCu's output layer) agrees with the
    GEMM-epilogue update + column-sum bias update it replaces"""
    x, e = rnd((1, n_in), 40), rnd((1, n_out), 41, 0.01)
    W, corr, b, corr_b = rnd((n_in, n_out), 42, 0.1), rnd((n_in, n_out), 43, 0.01), rnd(n_out, 44), rnd(n_out, 45)
    scale, l2 = -0.02, -1e-4
    out = []
    for fused in (True, False):
        dX, dE, dW, db = (DeviceArray.from_numpy(x), DeviceArray.from_numpy(e), DeviceArray.from_numpy(W),
                          DeviceArray.vector(b))
        dC = DeviceArray.from_numpy(corr) if mmt else None
        dCb = DeviceArray.vector(corr_b) if mmt else None
        if fused:
            check(lib().tnet_affine_update_row(dX.ptr, n_in, dE.ptr, n_out, dW.ptr, dW.stride,
                                               dC.ptr if dC else None, dC.stride if dC else 0, db.ptr,
                                               dCb.ptr if dCb else None, scale, mmt, l2, S()))
        else:
            ws = DeviceArray(1, max(1, lib().tnet_col_sum_workspace(dE.dim) // 4 + 64))
            check(lib().tnet_bias_update(dE.ptr, dE.dim, db.ptr, dCb.ptr if dCb else None, None, scale, mmt,
                                         ws.ptr, S()))
            check(lib().tnet_affine_update(dX.ptr, dX.dim, dE.ptr, dE.dim, dW.ptr, dW.dim, dC.ptr if dC else None,
                                           dC.stride if dC else 0, scale, mmt, l2, S()))
        synchronize()
        out.append([a.numpy() for a in (dW, db, dC, dCb) if a is not None])
    c = x.T.astype(np.float64) * e + mmt * corr
    w = W + scale * c
    w = w + l2 * w
    np.testing.assert_allclose(out[0][0], w, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(out[0][1].ravel(), b + scale * (e[0] + mmt * corr_b), rtol=1e-6, atol=1e-7)
    for a, r in zip(out[0], out[1]):
        np.testing.assert_allclose(a, r, rtol=2.5e-7, atol=1e-9)


def test_affine_update_row_rejects_missing_momentum_buffer():
    d = DeviceArray(1, 8)
    assert lib().tnet_affine_update_row(d.ptr, 8, d.ptr, 8, d.ptr, 8, None, 0, d.ptr, None, 0.1, 0.5, 0.0,
                                        S()) == -1  # TNET_ERR_ARG


class SgdSeg(C.Structure):
    _fields_ = [("p", C.c_void_p), ("g", C.c_void_p), ("corr", C.c_void_p), ("n", C.c_long), ("l2", C.c_float)]


@pytest.mark.parametrize("mmt", [0.0, 0.9])
@pytest.mark.parametrize("sizes", [[1], [4194304, 2048], [7, 13, 4096, 1, 5, 3, 1000, 9, 17, 4]])
def test_sgd_update_multi(mmt, sizes):
    """several SGD segments in one launch (more than 8 split over launches), ragged and unaligned sizes"""
    scale = -0.01
    segs, refs = [], []
    keep = []
    for k, n in enumerate(sizes):
        p, g, c = rnd(n, 30 + k), rnd(n, 50 + k), rnd(n, 70 + k, 0.1)
        l2 = -1e-4 * (k % 3)
        dp_, dg, dc = DeviceArray.vector(p), DeviceArray.vector(g), DeviceArray.vector(c)
        keep += [dp_, dg, dc]
        segs.append(SgdSeg(dp_.ptr, dg.ptr, dc.ptr if mmt else None, n, l2))
        cc = g.astype(np.float64) + mmt * c if mmt else g.astype(np.float64)
        w = p + scale * cc
        w = w + l2 * w
        refs.append((dp_, dc, w, cc))
    arr = (SgdSeg * len(segs))(*segs)
    check(lib().tnet_sgd_update_multi(C.cast(arr, C.c_void_p), len(segs), scale, mmt, S()))
    for dp_, dc, w, cc in refs:
        np.testing.assert_allclose(dp_.numpy().ravel(), w, rtol=1e-6, atol=1e-7)
        if mmt:
            np.testing.assert_allclose(dc.numpy().ravel(), cc, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("rows,cols", [(1, 1), (16, 10), (1024, 135), (1024, 4000), (300, 4099), (64, 5000)])
def test_softmax_xent_labels(rows, cols):
    Z = rnd((rows, cols), 16, 3.0)
    lab = np.random.default_rng(17).integers(0, cols, size=rows).astype(np.int32)
    lab[::7] = -1  # unlabeled frames: all-zero target rows
    dZ, dL = DeviceArray.from_numpy(Z), DeviceArray.vector(lab)
    dY, dE = DeviceArray(rows, cols), DeviceArray(rows, cols)
    stats = DeviceArray(1, 1024, np.float64, stride=1024)
    check(lib().tnet_softmax_xent(dZ.ptr, dZ.dim, dL.ptr, dY.ptr, dY.stride, dE.ptr, dE.stride, stats.ptr, S()))
    Yref = orc.softmax(Z)
    Eref, xent, correct = orc.xent_eval(Yref, lab)
    np.testing.assert_allclose(dY.numpy(), Yref, rtol=2e-5, atol=1e-9)
    np.testing.assert_allclose(dE.numpy(), Eref, rtol=2e-5, atol=1e-8)
    s = stats.numpy()[0]
    np.testing.assert_allclose(s[0::2].sum(), xent, rtol=1e-5, atol=1e-5)
    assert int(round(s[1::2].sum())) == correct


@pytest.mark.parametrize("rows,cols", [(64, 135), (64, 4000)])
def test_softmax_xent_label_out_of_range_is_unlabeled(rows, cols):
    """a class id >= N never indexes past the row: the kernels (both the one-wave-per-row and the
    four-waves-per-row form) treat it as an unlabeled row, like -1 (the host intake rejects it)"""
    Z = rnd((rows, cols), 21, 3.0)
    lab = np.random.default_rng(22).integers(0, cols, size=rows).astype(np.int32)
    bad = lab.copy()
    bad[::3] = cols
    bad[1::5] = cols + 1000
    ref = lab.copy()
    ref[bad >= cols] = -1
    out = []
    for L in (bad, ref):
        dZ, dL = DeviceArray.from_numpy(Z), DeviceArray.vector(L)
        dE = DeviceArray(rows, cols)
        stats = DeviceArray(1, 1024, np.float64, stride=1024)
        check(lib().tnet_softmax_xent(dZ.ptr, dZ.dim, dL.ptr, None, 0, dE.ptr, dE.stride, stats.ptr, S()))
        out.append((dE.numpy(), stats.numpy()[0]))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])


def test_softmax_xent_extreme_logits():
    """underflowing probabilities hit the FLT_MIN clamp of _log_elem (cukernels.cu:131-141)"""
    rows, cols = 8, 300
    Z = np.zeros((rows, cols), np.float32)
    Z[:, 0] = 200.0
    lab = np.full(rows, 5, np.int32)
    dZ, dL = DeviceArray.from_numpy(Z), DeviceArray.vector(lab)
    dE = DeviceArray(rows, cols)
    stats = DeviceArray(1, 1024, np.float64, stride=1024)
    check(lib().tnet_softmax_xent(dZ.ptr, dZ.dim, dL.ptr, None, 0, dE.ptr, dE.stride, stats.ptr, S()))
    e, c = C.c_double(), C.c_double()
    check(lib().tnet_stats_fetch(stats.ptr, C.byref(e), C.byref(c), S()))
    np.testing.assert_allclose(e.value, -rows * np.log(np.float32(1.1754944e-38)), rtol=1e-6)
    assert c.value == 0


@pytest.mark.parametrize("rows,cols", [(1, 1), (1024, 2048), (960, 135), (3, 4000), (2049, 77)])
def test_col_sum_and_bias_update(rows, cols):
    E = rnd((rows, cols), 18)
    dE = DeviceArray.from_numpy(E)
    v0 = rnd(cols, 19)
    dv = DeviceArray.vector(v0)
    ws = DeviceArray(1, max(1, lib().tnet_col_sum_workspace(dE.dim) // 4 + 64))
    check(lib().tnetF_add_col_sum(0.5, dE.ptr, 2.0, dv.ptr, dE.dim, ws.ptr, S()))
    ref = 0.5 * E.astype(np.float64).sum(0) + 2.0 * v0
    np.testing.assert_allclose(dv.numpy()[:, 0], ref, rtol=1e-5, atol=1e-5)
    # bias update with momentum
    b0, cb0 = rnd(cols, 20), rnd(cols, 21)
    db, dcb = DeviceArray.vector(b0), DeviceArray.vector(cb0)
    check(lib().tnet_bias_update(dE.ptr, dE.dim, db.ptr, dcb.ptr, None, -0.01, 0.9, ws.ptr, S()))
    c = E.astype(np.float64).sum(0) + 0.9 * cb0
    np.testing.assert_allclose(dcb.numpy()[:, 0], c, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(db.numpy()[:, 0], b0 - 0.01 * c, rtol=1e-5, atol=1e-6)


def test_elementwise_ops():
    rows, cols = 37, 131
    X = rnd((rows, cols), 22)
    Y = 1 / (1 + np.exp(-rnd((rows, cols), 23)))
    dX, dY, dO = DeviceArray.from_numpy(X), DeviceArray.from_numpy(Y), DeviceArray(rows, cols)
    check(lib().tnetF_sigmoid(dO.ptr, dX.ptr, dX.dim, S()))
    np.testing.assert_allclose(dO.numpy(), orc.sigmoid(X), rtol=2e-6, atol=1e-7)
    check(lib().tnetF_diff_sigmoid(dO.ptr, dX.ptr, dY.ptr, dX.dim, S()))
    np.testing.assert_allclose(dO.numpy(), orc.diff_sigmoid(X, Y), rtol=2e-6, atol=1e-7)
    r = rnd(cols, 24)
    dr = DeviceArray.vector(r)
    check(lib().tnetF_add_scaled_row(2.0, dr.ptr, 0.5, dX.ptr, dX.dim, S()))
    np.testing.assert_allclose(dX.numpy(), 2.0 * r + 0.5 * X, rtol=1e-6, atol=1e-6)
    check(lib().tnetF_set_const(dO.ptr, 3.5, dO.dim, S()))
    assert np.all(dO.numpy() == 3.5)
    P = np.abs(rnd((rows, cols), 25)) + 1e-3
    P[0, 0] = 0.0
    dP = DeviceArray.from_numpy(P)
    check(lib().tnetF_log_elem(dP.ptr, dP.dim, S()))
    ref = np.log(np.maximum(P, np.float32(1.1754944e-38)).astype(np.float64))
    np.testing.assert_allclose(dP.numpy(), ref, rtol=2e-6, atol=2e-6)


def test_randomize_and_gather():
    rows, cols = 500, 440
    X = rnd((rows, cols), 26)
    lab = np.arange(rows, dtype=np.int32) * 3
    perm = np.random.default_rng(27).permutation(rows).astype(np.int32)[:256]
    dX, dP, dL = DeviceArray.from_numpy(X), DeviceArray.vector(perm), DeviceArray.vector(lab)
    dY, dLo = DeviceArray(256, cols), DeviceArray.vector(np.zeros(256, np.int32))
    check(lib().tnetF_randomize(dY.ptr, dX.ptr, dP.ptr, dY.dim, dX.dim, S()))
    check(lib().tnet_gather_i32(dLo.ptr, dL.ptr, dP.ptr, 256, S()))
    np.testing.assert_array_equal(dY.numpy(), X[perm])
    np.testing.assert_array_equal(dLo.numpy()[:, 0], lab[perm])
    # both in one launch (the cache's GetBunchLabels)
    dY2, dLo2 = DeviceArray(256, cols), DeviceArray.vector(np.zeros(256, np.int32))
    check(lib().tnet_gather_bunch(dY2.ptr, dX.ptr, dLo2.ptr, dL.ptr, dP.ptr, dY2.dim, dX.dim, S()))
    np.testing.assert_array_equal(dY2.numpy(), X[perm])
    np.testing.assert_array_equal(dLo2.numpy()[:, 0], lab[perm])


@pytest.mark.parametrize("rows,cols", [(16, 10), (1000, 4000), (1024, 135), (33, 7)])
def test_colsum_slab_sums(rows, cols):
    E = rnd((rows, cols), 40)
    dE = DeviceArray.from_numpy(E)
    slabs = lib().tnet_colsum_slabs(rows)
    dP = DeviceArray.from_numpy(np.full((slabs, cols), np.nan, np.float32))
    check(lib().tnet_colsum_slab_sums(dE.ptr, dE.dim, dP.ptr, dP.stride, S()))
    P = dP.numpy()
    assert not np.isnan(P).any()
    # contract: tnet_colsum_slabs(rows) slabs of disjoint row ranges (the kernel's own boundaries when
    # rows is not a multiple of 32) whose sum is the column sum
    tot = np.abs(E).astype(np.float64).sum(0)
    assert np.all(np.abs(P.astype(np.float64).sum(0) - E.astype(np.float64).sum(0)) <= 32 * 1.2e-7 * tot + 1e-7)
    if rows % 32 == 0:
        assert np.all(np.abs(P - slab_sums(E)) <= 32 * 1.2e-7 * slab_sums(np.abs(E)) + 1e-7)


def test_check_class_first_max_wins():
    out = np.array([[0.1, 0.5, 0.5, 0.2], [0.3, 0.3, 0.3, 0.3], [0, 0, 0, 1]], np.float32)
    des = np.array([[0, 1, 0, 0], [1, 0, 0, 0], [0, 0, 1, 0]], np.float32)
    dO, dD = DeviceArray.from_numpy(out), DeviceArray.from_numpy(des, stride=DeviceArray.from_numpy(out).stride)
    m = DeviceArray.vector(np.zeros(3, np.int32))
    check(lib().tnetF_check_class(dO.ptr, dD.ptr, m.ptr, dO.dim, S()))
    np.testing.assert_array_equal(m.numpy()[:, 0], [1, 1, 0])


@pytest.mark.parametrize("mmt", [0.0, 0.5])
@pytest.mark.parametrize("rows,a_in,a_out,b_in,b_out", [(1024, 1024, 135, 598, 1024), (1024, 256, 135, 440, 256),
                                                        (512, 1024, 2048, 440, 2048)])
def test_affine_update_bias_pair(mmt, rows, a_in, a_out, b_in, b_out):
    """tnet_affine_update_bias_pair (two layers' fused weight + bias SGD in one launch, both on the 64x64
    configuration): each layer's W, momentum, b against the fp64 formula with tnet_affine_update_bias's
    tolerance; TNET_ERR_UNSUPPORTED when the two grids exceed one round over the CUs (the last case)"""
    scale, l2 = -0.3 / rows, -1e-4
    sides = []
    for k, (n_in, n_out) in enumerate([(a_in, a_out), (b_in, b_out)]):
        X, E = rnd((rows, n_in), 40 + k), rnd((rows, n_out), 50 + k, 0.01)
        W, corr = rnd((n_in, n_out), 60 + k, 0.1), rnd((n_in, n_out), 70 + k, 0.01)
        b, corr_b = rnd(n_out, 80 + k), rnd(n_out, 90 + k, 0.01)
        P = slab_sums(E).astype(np.float32)
        d = dict(X=X, E=E, W=W, corr=corr, b=b, corr_b=corr_b, P=P, dX=DeviceArray.from_numpy(X),
                 dE=DeviceArray.from_numpy(E), dW=DeviceArray.from_numpy(W), dP=DeviceArray.from_numpy(P),
                 db=DeviceArray.vector(b), dC=DeviceArray.from_numpy(corr) if mmt else None,
                 dCb=DeviceArray.vector(corr_b) if mmt else None)
        sides.append(d)
    args = []
    for d in sides:
        args += [d["dX"].ptr, d["dX"].dim, d["dE"].ptr, d["dE"].dim, d["dW"].ptr, d["dW"].dim,
                 d["dC"].ptr if d["dC"] else None, d["dC"].stride if d["dC"] else 0, scale, mmt, l2, d["dP"].ptr,
                 d["dP"].stride, d["db"].ptr, d["dCb"].ptr if d["dCb"] else None]
    st = lib().tnet_affine_update_bias_pair(*args, S())
    n_tiles = sum(-(-n_in // 64) * -(-n_out // 64) for n_in, n_out in [(a_in, a_out), (b_in, b_out)])
    if n_tiles > 256:
        assert st == -4  # TNET_ERR_UNSUPPORTED
        return
    check(st)
    for d in sides:
        g, mag = gemm_ref("T", "N", d["X"], d["E"])
        c = g + mmt * d["corr"]
        w = d["W"] + scale * c
        w = w + l2 * w
        tol = 2e-5 * abs(scale) * mag + 2e-7 * np.abs(d["W"]) + 1e-7
        assert np.all(np.abs(d["dW"].numpy() - w) <= tol)
        if mmt:
            assert np.all(np.abs(d["dC"].numpy() - c) <= 2e-5 * mag + 1e-6)
        gb = d["P"].astype(np.float64).sum(0).astype(np.float32).astype(np.float64)
        cb = gb + mmt * d["corr_b"]
        np.testing.assert_allclose(d["db"].numpy().ravel(), d["b"] + scale * cb, rtol=1e-6, atol=1e-7)
        if mmt:
            np.testing.assert_allclose(d["dCb"].numpy().ravel(), cb, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("mmt", [0.0, 0.5])
@pytest.mark.parametrize("rows,sides,gcols", [
    (1024, [(440, 2048)], 440),                  # dnn4's first-layer update (the step's last launch)
    (1024, [(598, 1024)], 598),                  # MLP3's first layer alone; 598 columns: 16-B pieces over 600
    (1024, [(1024, 135), (598, 1024)], 598),     # MLP3's last two updates (the pair)
    (256, [(440, 256)], 440),
    (1024, [(2048, 2048)], 440),                 # 128x128 alone: declined
    (1024, [(2048, 2048), (440, 2048)], 440),    # dnn4's last two updates: 128x128 direct + 64x64 (mixed kernel)
])
def test_affine_update_bias_gather_matches_separate_calls(mmt, rows, sides, gcols):
    """tnet_affine_update_bias_gather (the step's last weight update(s) + the next bunch's gather in ONE launch)
    against tnet_affine_update_bias / _pair followed by tnet_gather_bunch: W, momentum, b and its momentum
    bit-identical, the gathered rows and class ids exact; TNET_ERR_UNSUPPORTED where the update alone would
    run another tile configuration"""
    scale, l2 = -0.3 / rows, -1e-4
    cache_rows = 3000
    Xc = rnd((cache_rows, gcols), 300)
    labc = (np.arange(cache_rows, dtype=np.int32) * 7) % 4000
    perm = np.random.default_rng(301).permutation(cache_rows).astype(np.int32)[:1024]
    host = []
    for k, (n_in, n_out) in enumerate(sides):
        X, E = rnd((rows, n_in), 310 + k), rnd((rows, n_out), 320 + k, 0.01)
        W, corr = rnd((n_in, n_out), 330 + k, 0.1), rnd((n_in, n_out), 340 + k, 0.01)
        b, corr_b = rnd(n_out, 350 + k), rnd(n_out, 360 + k, 0.01)
        host.append((X, E, W, corr, b, corr_b, slab_sums(E).astype(np.float32)))
    results = []
    for fused in (True, False):
        dev, args = [], []
        for X, E, W, corr, b, corr_b, P in host:
            d = dict(dX=DeviceArray.from_numpy(X), dE=DeviceArray.from_numpy(E), dW=DeviceArray.from_numpy(W),
                     dP=DeviceArray.from_numpy(P), db=DeviceArray.vector(b),
                     dC=DeviceArray.from_numpy(corr) if mmt else None, dCb=DeviceArray.vector(corr_b) if mmt else None)
            dev.append(d)
            args.append([d["dX"].ptr, d["dX"].dim, d["dE"].ptr, d["dE"].dim, d["dW"].ptr, d["dW"].dim,
                         d["dC"].ptr if d["dC"] else None, d["dC"].stride if d["dC"] else 0, scale, mmt, l2,
                         d["dP"].ptr, d["dP"].stride, d["db"].ptr, d["dCb"].ptr if d["dCb"] else None])
        dXc, dLc, dPerm = DeviceArray.from_numpy(Xc), DeviceArray.vector(labc), DeviceArray.vector(perm)
        dY = DeviceArray.from_numpy(np.full((1024, gcols), np.nan, np.float32))
        dLo = DeviceArray.vector(np.full(1024, -7, np.int32))
        gargs = [dY.ptr, dXc.ptr, dLo.ptr, dLc.ptr, dPerm.ptr, dY.dim, dXc.dim]
        if fused:
            second = args[1] if len(args) > 1 else [None, MatrixDim(0, 0, 0), None, MatrixDim(0, 0, 0), None,
                                                     MatrixDim(0, 0, 0), None, 0, 0.0, 0.0, 0.0, None, 0, None, None]
            # a destination inside the update's own X: refused before anything is launched
            bad = [dev[0]["dX"].ptr, dXc.ptr, dLo.ptr, dLc.ptr, dPerm.ptr, MatrixDim(8, gcols, dev[0]["dX"].stride),
                   dXc.dim]
            if dev[0]["dX"].cols == gcols:
                assert lib().tnet_affine_update_bias_gather(*args[0], *second, *bad, S()) == TNET_ERR_ARG
            st = lib().tnet_affine_update_bias_gather(*args[0], *second, *gargs, S())
            if sides == [(2048, 2048)]:
                assert st == TNET_ERR_UNSUPPORTED
                return
            check(st)
        else:
            if len(args) > 1:
                st2 = lib().tnet_affine_update_bias_pair(*args[0], *args[1], S())
                if st2 == TNET_ERR_UNSUPPORTED:  # grids in two configurations: the two separate calls
                    for a in args:
                        check(lib().tnet_affine_update_bias(*a, S()))
                else:
                    check(st2)
            else:
                for a in args:
                    check(lib().tnet_affine_update_bias(*a, S()))
            check(lib().tnet_gather_bunch(*gargs, S()))
        out = []
        for d in dev:
            out += [d["dW"].numpy(), d["db"].numpy()]
            if mmt:
                out += [d["dC"].numpy(), d["dCb"].numpy()]
        results.append((out, dY.numpy(), dLo.numpy()[:, 0]))
    (oa, ya, la), (ob, yb, lb) = results
    for a, b_ in zip(oa, ob):
        np.testing.assert_array_equal(a, b_)
    np.testing.assert_array_equal(ya, Xc[perm])
    np.testing.assert_array_equal(yb, Xc[perm])
    np.testing.assert_array_equal(la, labc[perm])
    np.testing.assert_array_equal(lb, labc[perm])


@pytest.mark.parametrize("rows,n_in,n_out,gcols", [(1024, 440, 2048, 440), (1024, 598, 1024, 598), (256, 440, 256, 440),
                                                  (1024, 2048, 2048, 440)])
def test_affine_grad_bias_gather_matches_separate_calls(rows, n_in, n_out, gcols):
    """tnet_affine_grad_bias_gather (the data-parallel step's last gradient GEMM + the next bunch's gather in ONE
    launch) against tnet_affine_grad_bias followed by tnet_gather_bunch: G and the bias gradient bit-identical, the
    gathered rows and class ids exact; TNET_ERR_UNSUPPORTED where the GEMM alone runs another tile configuration"""
    cache_rows = 3000
    Xc = rnd((cache_rows, gcols), 500)
    labc = (np.arange(cache_rows, dtype=np.int32) * 7) % 4000
    perm = np.random.default_rng(501).permutation(cache_rows).astype(np.int32)[:1024]
    X, E = rnd((rows, n_in), 510), rnd((rows, n_out), 520, 0.01)
    P = slab_sums(E).astype(np.float32)
    dX, dE, dP = DeviceArray.from_numpy(X), DeviceArray.from_numpy(E), DeviceArray.from_numpy(P)
    results = []
    for fused in (True, False):
        dG = DeviceArray.from_numpy(np.full((n_in, n_out), np.nan, np.float32))
        dgb = DeviceArray.vector(np.full(n_out, np.nan, np.float32))
        dXc, dLc, dPerm = DeviceArray.from_numpy(Xc), DeviceArray.vector(labc), DeviceArray.vector(perm)
        dY = DeviceArray.from_numpy(np.full((1024, gcols), np.nan, np.float32))
        dLo = DeviceArray.vector(np.full(1024, -7, np.int32))
        gargs = [dY.ptr, dXc.ptr, dLo.ptr, dLc.ptr, dPerm.ptr, dY.dim, dXc.dim]
        args = [dX.ptr, dX.dim, dE.ptr, dE.dim, dG.ptr, dG.dim, dP.ptr, dP.stride, dgb.ptr]
        if fused:
            nil = [None, MatrixDim(0, 0, 0), None, MatrixDim(0, 0, 0), None, MatrixDim(0, 0, 0), None, 0, None]
            st = lib().tnet_affine_grad_bias_gather(*args, *nil, *gargs, S())
            if n_in == 2048:
                assert st == TNET_ERR_UNSUPPORTED
                return
            check(st)
        else:
            check(lib().tnet_affine_grad_bias(*args, S()))
            check(lib().tnet_gather_bunch(*gargs, S()))
        results.append((dG.numpy(), dgb.numpy(), dY.numpy(), dLo.numpy()[:, 0]))
    (ga, ba, ya, la), (gb_, bb, yb, lb) = results
    np.testing.assert_array_equal(ga, gb_)
    np.testing.assert_array_equal(ba, bb)
    np.testing.assert_allclose(ga, X.astype(np.float64).T @ E.astype(np.float64), rtol=1e-4, atol=1e-5)
    for y_, l_ in ((ya, la), (yb, lb)):
        np.testing.assert_array_equal(y_, Xc[perm])
        np.testing.assert_array_equal(l_, labc[perm])


def test_affine_grad_bias_gather_two_gemms_mlp3():
    """the two-GEMM form of tnet_affine_grad_bias_gather on MLP3's last two gradients (598x1024 over the bunch, and
    1024x135 -- which the planner alone would split over K): both gradients and bias gradients against the fp64
    products (each GEMM unsplit here, its sums in k order: bit-identical to the single form where that runs unsplit
    too, within fp32 summation order of a split-K run otherwise), the gathered rows and class ids exact"""
    rows = 1024
    X1, E1 = rnd((rows, 598), 530), rnd((rows, 1024), 531, 0.01)
    X2, E2 = rnd((rows, 1024), 532), rnd((rows, 135), 533, 0.01)
    P1, P2 = slab_sums(E1).astype(np.float32), slab_sums(E2).astype(np.float32)
    Xc = rnd((3000, 598), 534)
    labc = (np.arange(3000, dtype=np.int32) * 7) % 135
    perm = np.random.default_rng(535).permutation(3000).astype(np.int32)[:rows]
    d = {k: DeviceArray.from_numpy(v) for k, v in dict(X1=X1, E1=E1, X2=X2, E2=E2, P1=P1, P2=P2, Xc=Xc).items()}
    dG1 = DeviceArray.from_numpy(np.full((598, 1024), np.nan, np.float32))
    dG2 = DeviceArray.from_numpy(np.full((1024, 135), np.nan, np.float32))
    db1, db2 = DeviceArray.vector(np.full(1024, np.nan, np.float32)), DeviceArray.vector(np.full(135, np.nan, np.float32))
    dLc, dPerm = DeviceArray.vector(labc), DeviceArray.vector(perm)
    dY = DeviceArray.from_numpy(np.full((rows, 598), np.nan, np.float32))
    dLo = DeviceArray.vector(np.full(rows, -7, np.int32))
    st = lib().tnet_affine_grad_bias_gather(
        d["X2"].ptr, d["X2"].dim, d["E2"].ptr, d["E2"].dim, dG2.ptr, dG2.dim, d["P2"].ptr, d["P2"].stride, db2.ptr,
        d["X1"].ptr, d["X1"].dim, d["E1"].ptr, d["E1"].dim, dG1.ptr, dG1.dim, d["P1"].ptr, d["P1"].stride, db1.ptr,
        dY.ptr, d["Xc"].ptr, dLo.ptr, dLc.ptr, dPerm.ptr, dY.dim, d["Xc"].dim, S())
    if st == TNET_ERR_UNSUPPORTED:
        pytest.skip("the pair does not fit one round on this device")
    check(st)
    for G, b, X, E, P in ((dG1, db1, X1, E1, P1), (dG2, db2, X2, E2, P2)):
        np.testing.assert_allclose(G.numpy(), X.astype(np.float64).T @ E.astype(np.float64), rtol=1e-4, atol=1e-5)
        np.testing.assert_array_equal(b.numpy().ravel(), P.astype(np.float64).sum(0).astype(np.float32))
    np.testing.assert_array_equal(dY.numpy(), Xc[perm])
    np.testing.assert_array_equal(dLo.numpy()[:, 0], labc[perm])


@pytest.mark.parametrize("rows,n_in,n_out", [(1024, 2048, 4000), (1024, 2048, 2048), (256, 512, 1000), (64, 128, 4000)])
def test_affine_bwd_colsum_slabs_matches_two_calls(rows, n_in, n_out):
    """tnet_affine_bwd_colsum_slabs (the top layer's backward GEMM + the slab sums of its input error in ONE
    launch) against tnet_colsum_slab_sums + tnet_affine_bwd_colsum: Eo, Eo's slab sums and E's slab sums bit
    for bit; TNET_ERR_UNSUPPORTED where the backward alone would run another tile configuration"""
    E = rnd((rows, n_out), 400, 0.01)
    W = rnd((n_in, n_out), 401, 0.05)
    Yb = np.random.default_rng(402).random((rows, n_in)).astype(np.float32)
    slabs = lib().tnet_colsum_slabs(rows)
    dE, dW, dY = DeviceArray.from_numpy(E), DeviceArray.from_numpy(W), DeviceArray.from_numpy(Yb)
    out = []
    for one in (True, False):
        dEo = DeviceArray.from_numpy(np.full((rows, n_in), np.nan, np.float32))
        dP = DeviceArray.from_numpy(np.full((slabs, n_in), np.nan, np.float32))
        dPt = DeviceArray.from_numpy(np.full((slabs, n_out), np.nan, np.float32))
        if one:
            st = lib().tnet_affine_bwd_colsum_slabs(dE.ptr, dE.dim, dW.ptr, dW.dim, dY.ptr, dY.stride, dEo.ptr, dEo.dim,
                                                    dP.ptr, dP.stride, dPt.ptr, dPt.stride, S())
            if -(-rows // 64) * -(-n_in // 128) < 200:
                assert st == TNET_ERR_UNSUPPORTED
                return
            check(st)
        else:
            check(lib().tnet_colsum_slab_sums(dE.ptr, dE.dim, dPt.ptr, dPt.stride, S()))
            check(lib().tnet_affine_bwd_colsum(dE.ptr, dE.dim, dW.ptr, dW.dim, dY.ptr, dY.stride, dEo.ptr, dEo.dim,
                                               dP.ptr, dP.stride, S()))
        out.append((dEo.numpy(), dP.numpy(), dPt.numpy()))
    for a, b in zip(out[0], out[1]):
        assert not np.isnan(a).any()
        np.testing.assert_array_equal(a, b)
    np.testing.assert_allclose(out[0][2], slab_sums(E), rtol=1e-5, atol=1e-6)
