#!/usr/bin/env python3
"""The backward GEMM (Eo = diff-sigmoid(E W^T), k-contiguous A = E and B = W) at 1024 x 2048 over K = 2048 with
the operands' row strides padded past the 8-KiB power of two, in the LDS ring form (m64x128k64s2) and the
coalesced direct form (m64x128c8): does the row stride, not the load pattern, hold the direct form back?
usage: python tools/gemm_stride_ab.py [iters]"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import numpy as np  # noqa: E402
from tnet_amd import DeviceArray  # noqa: E402
from tnet_amd._lib import lib, check  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
S = lib().tnet_stream()
rows, ni, no = 1024, 2048, 2048
rng = np.random.default_rng(0)
E = (0.01 * rng.standard_normal((rows, no))).astype(np.float32)
W = (0.05 * rng.standard_normal((ni, no))).astype(np.float32)
Yb = rng.random((rows, ni)).astype(np.float32)
out = []
ref = None
for pad in (0, 64, 128, 32):
    dE = DeviceArray.from_numpy(E, stride=no + pad)
    dW = DeviceArray.from_numpy(W, stride=no + pad)
    dY = DeviceArray.from_numpy(Yb)
    dO = DeviceArray(rows, ni)
    for cfg in ("m64x128k64s2", "m64x128c8"):
        check(lib().tnet_gemm_config(cfg.encode()))
        run = lambda: check(lib().tnet_affine_bwd(dE.ptr, dE.dim, dW.ptr, dW.dim, dY.ptr, dY.stride, dO.ptr, dO.dim, 1, S))
        for _ in range(3):
            run()
        ms = C.c_float()
        check(lib().tnet_timer_start())
        for _ in range(iters):
            run()
        check(lib().tnet_timer_stop(C.byref(ms)))
        o = dO.numpy()
        same = bool(ref is None or np.array_equal(o, ref))
        ref = o if ref is None else ref
        us = 1000.0 * ms.value / iters
        out.append({"cfg": cfg, "row_stride_floats": no + pad, "us": round(us, 2),
                    "tflops": round(2.0 * rows * ni * no / (us * 1e-6) / 1e12, 1), "bit_identical": same})
        print(json.dumps(out[-1]), flush=True)
check(lib().tnet_gemm_config(b"auto"))
print("RESULT " + json.dumps(out))
