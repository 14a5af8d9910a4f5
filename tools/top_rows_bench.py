#!/usr/bin/env python3
"""Launch-level timing of the narrow top layer (BASELINE config 2: 1024 x 1024 -> 135): tnet_affine_fwd (logits) and
tnet_affine_softmax_xent (logits + softmax + xent + error + slab sums), back-to-back launches on the library stream,
wall clock over `reps` launches after a warm-up (launch gaps included).  Run with TNET_TOP_SPLIT=0 for the general
GEMM's split-K form.  Prints one JSON line.

usage: python tools/top_rows_bench.py [--rows 1024] [--n-in 1024] [--n-out 135] [--reps 400]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import numpy as np  # noqa: E402

from tnet_amd import DeviceArray, synchronize  # noqa: E402
from tnet_amd._lib import check, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1024)
    ap.add_argument("--n-in", type=int, default=1024)
    ap.add_argument("--n-out", type=int, default=135)
    ap.add_argument("--reps", type=int, default=400)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    X = DeviceArray.from_numpy(rng.random((a.rows, a.n_in), dtype=np.float32))
    W = DeviceArray.from_numpy((0.05 * rng.standard_normal((a.n_in, a.n_out))).astype(np.float32))
    b = DeviceArray.vector(np.zeros(a.n_out, np.float32))
    L = DeviceArray.vector(rng.integers(0, a.n_out, a.rows).astype(np.int32))
    Z, E = DeviceArray(a.rows, a.n_out), DeviceArray(a.rows, a.n_out)
    stats = DeviceArray(1, 1024, np.float64, stride=1024)
    P = DeviceArray(lib().tnet_colsum_slabs(a.rows), a.n_out)
    S = lib().tnet_stream()

    def fwd():
        check(lib().tnet_affine_fwd(X.ptr, X.dim, W.ptr, W.dim, b.ptr, Z.ptr, Z.dim, 0, S))

    def fused():
        check(lib().tnet_affine_softmax_xent(X.ptr, X.dim, W.ptr, W.dim, b.ptr, L.ptr, Z.ptr, Z.stride, None, 0, E.ptr,
                                             E.stride, stats.ptr, P.ptr, P.stride, S))

    out = {"rows": a.rows, "n_in": a.n_in, "n_out": a.n_out, "reps": a.reps,
           "top_split": os.environ.get("TNET_TOP_SPLIT", "1")}
    for name, fn in (("affine_fwd", fwd), ("affine_softmax_xent", fused)):
        for _ in range(50):
            fn()
        synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        synchronize()
        out[name + "_us"] = round(1e6 * (time.perf_counter() - t0) / a.reps, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
