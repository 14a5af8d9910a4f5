#!/usr/bin/env python3
"""Sweep the GEMM tile configurations (TNET_GEMM_CFG; "auto" = the library's own choice; a "+sk<n>"
suffix forces a split-K count, TNET_GEMM_SPLITK) over the SGD-step shapes on the GPU.

Each configuration runs in its own process (the config is read once per process); every shape is
timed with hipEvents on the library stream over `iters` back-to-back launches of the FUSED kernels
the training step uses (affine fwd + sigmoid, affine bwd + diff-sigmoid, affine update + SGD; kinds
"bwdcs" / "updb" add the bias-gradient slab sums / the bias SGD, as CuNetwork's step calls them)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFGS = ["g64x64k32s4w4", "m64x128k64s2", "m128x128k64s2", "m128x256k32s3", "m64x64k64s2", "m64x64k32s4", "m32x64k64s2",
        "m64x64k32s4w41", "m64x128a4", "m64x128a8", "m128x128a4", "m128x256a2", "m64x64a4", "m64x128c8"]
# (kind, rows, n_in, n_out): fwd/bwd/upd of each layer of 440 -> 2048x4 -> 4000 at bunch 1024
SHAPES = [("fwd", 1024, 2048, 2048), ("bwd", 1024, 2048, 2048), ("upd", 1024, 2048, 2048),
          ("fwd", 1024, 2048, 4000), ("bwd", 1024, 2048, 4000), ("upd", 1024, 2048, 4000),
          ("fwd", 1024, 440, 2048), ("upd", 1024, 440, 2048)]

CHILD = r'''
import sys, json, ctypes as C
sys.path.insert(0, sys.argv[1] + "/nnet-asr_amd")
import numpy as np
from tnet_amd import DeviceArray
from tnet_amd._lib import lib, check
shapes = json.loads(sys.argv[2]); iters = int(sys.argv[3])
S = lib().tnet_stream()
out = []
for kind, rows, ni, no in shapes:
    rng = np.random.default_rng(0)
    X = DeviceArray.from_numpy(rng.standard_normal((rows, ni)).astype(np.float32))
    W = DeviceArray.from_numpy((0.05 * rng.standard_normal((ni, no))).astype(np.float32))
    E = DeviceArray.from_numpy((0.01 * rng.standard_normal((rows, no))).astype(np.float32))
    b = DeviceArray.vector(np.zeros(no, np.float32))
    Y = DeviceArray(rows, no)
    Eo = DeviceArray(rows, ni)
    slabs = lib().tnet_colsum_slabs(rows)
    Po = DeviceArray(slabs, ni)
    Pi = DeviceArray.from_numpy(np.zeros((slabs, no), np.float32))
    bb = DeviceArray.vector(np.zeros(no, np.float32))
    def run():
        if kind == "fwd":
            check(lib().tnet_affine_fwd(X.ptr, X.dim, W.ptr, W.dim, b.ptr, Y.ptr, Y.dim, 1, S))
        elif kind == "bwd":
            check(lib().tnet_affine_bwd(E.ptr, E.dim, W.ptr, W.dim, X.ptr, X.stride, Eo.ptr, Eo.dim, 1, S))
        elif kind == "bwdcs":  # the training step's bwd: + diff-sigmoid + slab column sums
            check(lib().tnet_affine_bwd_colsum(E.ptr, E.dim, W.ptr, W.dim, X.ptr, X.stride, Eo.ptr, Eo.dim, Po.ptr,
                                               Po.stride, S))
        elif kind == "updb":  # the training step's update: + the bias SGD from slab sums
            check(lib().tnet_affine_update_bias(X.ptr, X.dim, E.ptr, E.dim, W.ptr, W.dim, None, 0, -1e-6, 0.0, 0.0,
                                                Pi.ptr, Pi.stride, bb.ptr, None, S))
        else:
            check(lib().tnet_affine_update(X.ptr, X.dim, E.ptr, E.dim, W.ptr, W.dim, None, 0, -1e-6, 0.0, 0.0, S))
    for _ in range(3): run()
    ms = C.c_float()
    check(lib().tnet_timer_start())
    for _ in range(iters): run()
    check(lib().tnet_timer_stop(C.byref(ms)))
    us = 1000.0 * ms.value / iters
    out.append([kind, rows, ni, no, us, 2.0 * rows * ni * no / (us * 1e-6) / 1e12])
print("RESULT " + json.dumps(out))
'''


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    cfgs = sys.argv[2].split(",") if len(sys.argv) > 2 else CFGS
    shapes = json.loads(sys.argv[3]) if len(sys.argv) > 3 else SHAPES
    res = {}
    for cfg in cfgs:
        parts = cfg.split("+")
        env = dict(os.environ, TNET_GEMM_CFG=parts[0])
        for extra in parts[1:]:
            if extra == "noload":
                env["TNET_GEMM_DIAG"] = "1"
            elif extra.startswith("diag"):
                env["TNET_GEMM_DIAG"] = extra[4:]
            elif extra.startswith("g") and extra[1:].isdigit():
                env["TNET_GEMM_GROUP"] = extra[1:]
            elif extra.startswith("sk") and extra[2:].isdigit():
                env["TNET_GEMM_SPLITK"] = extra[2:]
            elif extra.startswith("split2_") and extra[7:].isdigit():
                env["TNET_GEMM_SPLIT2"] = extra[7:]  # gemm16_split2_kernel for the few-tile updates
        p = subprocess.run([sys.executable, "-c", CHILD, REPO, json.dumps(shapes), str(iters)], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
        if p.returncode != 0 or not line:
            print(cfg, "FAILED", p.stderr[-500:], flush=True)
            if p.returncode < 0 or p.returncode in (134, 139):
                break
            continue
        res[cfg] = json.loads(line[0][7:])
        for kind, rows, ni, no, us, tf in res[cfg]:
            print(f"{cfg:12s} {kind} {rows}x{ni}x{no}: {us:8.1f} us {tf:6.1f} TF/s", flush=True)
    print("SWEEP " + json.dumps(res))


if __name__ == "__main__":
    main()
