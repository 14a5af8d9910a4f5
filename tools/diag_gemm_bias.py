#!/usr/bin/env python3
"""Is the fp32 MFMA GEMM's rounding unbiased?  C = A B on the GPU (tnet_sgemm, every layout) vs the
fp64 product: the mean SIGNED magnitude error E[(|C| - |C64|) / |C64|] over all elements (a bias toward
zero shows as a negative mean many standard errors from 0), next to the same statistic for numpy's
fp32 matmul (MKL / OpenBLAS, round to nearest) on the same operands."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import numpy as np  # noqa: E402

import tnet_amd  # noqa: E402
from tnet_amd._lib import check, lib  # noqa: E402


def stats(C, R):
    m = np.abs(R) > 1e-3 * np.abs(R).mean()
    rel = (np.abs(C.astype(np.float64)) - np.abs(R))[m] / np.abs(R)[m]
    return rel.mean(), rel.std() / np.sqrt(rel.size), np.abs(rel).mean()


rng = np.random.default_rng(0)
for (M, N, K) in [(1024, 2048, 2048), (1024, 135, 1024), (598, 1024, 960), (1024, 1024, 598)]:
    for ta, tb in [("N", "N"), ("N", "T"), ("T", "N")]:
        A = rng.standard_normal((K, M) if ta == "T" else (M, K)).astype(np.float32)
        B = rng.standard_normal((N, K) if tb == "T" else (K, N)).astype(np.float32)
        dA, dB = tnet_amd.DeviceArray.from_numpy(A), tnet_amd.DeviceArray.from_numpy(B)
        dC = tnet_amd.DeviceArray(M, N)
        check(lib().tnet_sgemm(ta.encode(), tb.encode(), M, N, K, ctypes.c_float(1.0), dA.ptr, dA.dim.stride, dB.ptr,
                               dB.dim.stride, ctypes.c_float(0.0), dC.ptr, dC.dim.stride, lib().tnet_stream()),
              "sgemm")
        C = dC.numpy()
        a64 = (A.T if ta == "T" else A).astype(np.float64)
        b64 = (B.T if tb == "T" else B).astype(np.float64)
        R = a64 @ b64
        F = (A.T if ta == "T" else A) @ (B.T if tb == "T" else B)
        g = stats(C, R)
        c = stats(F, R)
        print(f"{M}x{N}x{K} {ta}{tb}: GPU mean signed rel {g[0]:+.3e} (+-{g[1]:.1e}) mean |rel| {g[2]:.3e} | "
              f"numpy fp32 {c[0]:+.3e} (+-{c[1]:.1e}) mean |rel| {c[2]:.3e}", flush=True)
