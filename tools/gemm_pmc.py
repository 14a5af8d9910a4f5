"""Drive one GEMM shape repeatedly for rocprofv3 --pmc passes: our fused affine kernels
(TNET_GEMM_CFG selects the tile config) and, for comparison, torch.mm (hipBLASLt) on the same
shapes and data distribution.

  ours   fwd only (1024 x 2048 x 2048, bias + sigmoid)
  layer  the bench's roofline kernel set: one 2048x2048 <biasedlinearity> layer's fwd (bias +
         sigmoid), bwd (diff-sigmoid) and fused SGD update per iteration, bunch 1024, exactly the
         launches bench.py times (momentum 0, weight cost 0 -> no momentum buffer); as the step runs a
         hidden layer since round 5, the update keeps the transposed shadow W^T and the backward reads
         it (NN; TNET_BWD_SHADOW=0: the NT backward from W)
  torch  torch.mm on the fwd shape

usage: python tools/gemm_pmc.py [ours|layer|torch] [iters]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import numpy as np  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "ours"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows, ni, no = 1024, 2048, 2048
if which == "ours":
    from tnet_amd import DeviceArray
    from tnet_amd._lib import check, lib
    S = lib().tnet_stream()
    rng = np.random.default_rng(0)
    X = DeviceArray.from_numpy(rng.standard_normal((rows, ni)).astype(np.float32))
    W = DeviceArray.from_numpy((0.05 * rng.standard_normal((ni, no))).astype(np.float32))
    b = DeviceArray.vector(np.zeros(no, np.float32))
    Y = DeviceArray(rows, no)
    for _ in range(iters):
        check(lib().tnet_affine_fwd(X.ptr, X.dim, W.ptr, W.dim, b.ptr, Y.ptr, Y.dim, 1, S))
    check(lib().tnet_synchronize())
elif which == "layer":
    from tnet_amd import DeviceArray
    from tnet_amd._lib import check, lib
    S = lib().tnet_stream()
    rng = np.random.default_rng(0)
    X = DeviceArray.from_numpy((1.0 / (1.0 + np.exp(-rng.standard_normal((rows, ni))))).astype(np.float32))
    W = DeviceArray.from_numpy((0.05 * rng.standard_normal((ni, no))).astype(np.float32))
    b = DeviceArray.vector(np.zeros(no, np.float32))
    Y = DeviceArray(rows, no)
    E = DeviceArray.from_numpy((1e-3 * rng.standard_normal((rows, no))).astype(np.float32))
    Eo = DeviceArray(rows, ni)
    # the training step's fused forms: bwd writes the bias gradient of the layer below as slab sums,
    # the update applies the bias SGD from slab sums
    slabs = lib().tnet_colsum_slabs(rows)
    Po = DeviceArray(slabs, ni)
    Pi = DeviceArray.from_numpy(np.zeros((slabs, no), np.float32))
    shadow = os.environ.get("TNET_BWD_SHADOW", "2") != "0"
    if shadow:
        Wt = DeviceArray(no, ni)
        check(lib().tnet_transpose(W.ptr, W.dim, Wt.ptr, Wt.stride, S))
        check(lib().tnet_weight_shadow(W.ptr, W.dim, Wt.ptr, Wt.stride))
    for _ in range(iters):
        check(lib().tnet_affine_fwd(X.ptr, X.dim, W.ptr, W.dim, b.ptr, Y.ptr, Y.dim, 1, S))
        if shadow:
            check(lib().tnet_affine_bwd_colsum_t(E.ptr, E.dim, Wt.ptr, Wt.dim, X.ptr, X.stride, Eo.ptr, Eo.dim,
                                                 Po.ptr, Po.stride, S))
        else:
            check(lib().tnet_affine_bwd_colsum(E.ptr, E.dim, W.ptr, W.dim, X.ptr, X.stride, Eo.ptr, Eo.dim, Po.ptr,
                                               Po.stride, S))
        check(lib().tnet_affine_update_bias(X.ptr, X.dim, E.ptr, E.dim, W.ptr, W.dim, None, 0, -1e-6, 0.0, 0.0,
                                            Pi.ptr, Pi.stride, b.ptr, None, S))
    check(lib().tnet_synchronize())
    if shadow:
        check(lib().tnet_weight_shadow(W.ptr, W.dim, None, 0))
else:
    import torch
    torch.backends.cuda.matmul.allow_tf32 = False
    a = torch.randn(rows, ni, device="cuda")
    w = 0.05 * torch.randn(ni, no, device="cuda")
    for _ in range(iters):
        c = a @ w
    torch.cuda.synchronize()
