#!/usr/bin/env python3
"""In-kernel clock and cycle split of the 16x16x4 GEMM (diagnostic; MI355X_MICROARCH.md 'DVFS give-back'
item 6).  Loads the clock-stamped build (make -C nnet-asr_amd stamp -> lib/libtnet_amd_stamp.so), runs the
bench's roofline kernel set (one 2048x2048 <biasedlinearity> layer: fwd + sigmoid, bwd + diff-sigmoid,
fused SGD update, bunch 1024) back to back for `warm_s` seconds, then times single stamped launches.

Per workgroup (wave 0): s_memtime at entry / after the prologue / after the main loop / after the
epilogue, s_memrealtime (100 MHz) at entry and exit.  Reports the median in-kernel clock, the cycle
split, the MFMA-issue floor of the main loop (MFMAs of one wave x 32 cycles) and the launch spread.

usage: python tools/gemm_clock.py [warm_s] [reps] [cfg|auto] [rows,n_in,n_out] [kinds]"""
import ctypes as C
import json
import os
import sys
import time

os.environ.setdefault("TNET_DIAG_STAMP_LIB", "1")  # or nodma / noread / nobar (ablation builds)
if len(sys.argv) > 3 and sys.argv[3] != "auto":
    os.environ["TNET_GEMM_CFG"] = sys.argv[3]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import numpy as np  # noqa: E402
from tnet_amd import DeviceArray  # noqa: E402
from tnet_amd._lib import check, lib  # noqa: E402

warm_s = float(sys.argv[1]) if len(sys.argv) > 1 else 1.5
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows, ni, no = (int(x) for x in sys.argv[4].split(",")) if len(sys.argv) > 4 else (1024, 2048, 2048)
KINDS = sys.argv[5].split(",") if len(sys.argv) > 5 else ["fwd", "bwd", "upd"]
L = lib()
L.tnet_diag_stamps.restype = C.c_int
L.tnet_diag_stamps.argtypes = [C.c_void_p, C.c_int]
S = L.tnet_stream()
rng = np.random.default_rng(0)
X = DeviceArray.from_numpy((1.0 / (1.0 + np.exp(-rng.standard_normal((rows, ni))))).astype(np.float32))
W = DeviceArray.from_numpy((0.05 * rng.standard_normal((ni, no))).astype(np.float32))
b = DeviceArray.vector(np.zeros(no, np.float32))
Y = DeviceArray(rows, no)
E = DeviceArray.from_numpy((1e-3 * rng.standard_normal((rows, no))).astype(np.float32))
Eo = DeviceArray(rows, ni)
Po = DeviceArray(L.tnet_colsum_slabs(rows), ni)
Pi = DeviceArray.from_numpy(np.zeros((L.tnet_colsum_slabs(rows), no), np.float32))


def run(kind):
    if kind == "fwd":
        check(L.tnet_affine_fwd(X.ptr, X.dim, W.ptr, W.dim, b.ptr, Y.ptr, Y.dim, 1, S))
    elif kind == "bwd":  # the training step's fused forms (bias gradient as slab sums)
        check(L.tnet_affine_bwd_colsum(E.ptr, E.dim, W.ptr, W.dim, X.ptr, X.stride, Eo.ptr, Eo.dim, Po.ptr,
                                       Po.stride, S))
    else:
        check(L.tnet_affine_update_bias(X.ptr, X.dim, E.ptr, E.dim, W.ptr, W.dim, None, 0, -1e-9, 0.0, 0.0, Pi.ptr,
                                        Pi.stride, b.ptr, None, S))


def warm():
    t0 = time.time()
    while time.time() - t0 < warm_s:
        for _ in range(30):
            for k in KINDS:
                run(k)
        check(L.tnet_synchronize())


out = {}
nwg = 256  # 64x128 / 128x128 tiles of the 2048x2048 layer at bunch 1024
buf = (C.c_ulonglong * (6 * 8192))()
for kind in KINDS:
    recs = []
    for _ in range(reps):
        warm()
        check(L.tnet_diag_stamps_clear())
        run(kind)
        check(L.tnet_synchronize())
        check(L.tnet_diag_stamps(C.addressof(buf), 8192))
        a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 6).astype(np.int64)
        n = int((a[:, 5] > a[:, 4]).sum())  # workgroups of this launch (grid may differ per config)
        a = a[:n]
        t0, t1, t2, t3, r0, r1 = (a[:, i] for i in range(6))
        clk = (t3 - t0) / np.maximum(r1 - r0, 1) * 0.1  # GHz (realtime = 100 MHz)
        recs.append(dict(n_wg=n, clock_GHz=float(np.median(clk)), prologue_cyc=float(np.median(t1 - t0)),
                         main_cyc=float(np.median(t2 - t1)), epilogue_cyc=float(np.median(t3 - t2)),
                         total_cyc=float(np.median(t3 - t0)),
                         total_cyc_max=float(np.max(t3 - t0)),
                         n_wg_slow=float(np.sum((t3 - t0) > np.median(t3 - t0) + 2000)),
                         end_rt_spread_us=float((np.percentile(r1, 100) - np.percentile(r1, 50)) / 100.0),
                         start_spread_us=float((r0.max() - r0.min()) / 100.0),
                         end_spread_us=float((r1.max() - r1.min()) / 100.0),
                         span_us=float((r1.max() - r0.min()) / 100.0)))
    med = {k: float(np.median([r[k] for r in recs])) for k in recs[0]}
    # MFMA floor of the main loop: one wave's 16x16x4 MFMAs x 32 cycles (4 waves, one per SIMD)
    n = int(med["n_wg"])
    mfma_per_wave = 2.0 * rows * ni * no / 2048.0 / n / 4.0
    med["mfma_floor_cyc"] = mfma_per_wave * 32.0
    med["main_mfma_util"] = med["mfma_floor_cyc"] / med["main_cyc"]
    med["total_mfma_util"] = med["mfma_floor_cyc"] / med["total_cyc"]
    out[kind] = med
    print(kind, json.dumps({k: round(v, 3) for k, v in med.items()}), flush=True)
print("CLOCK " + json.dumps(out))
