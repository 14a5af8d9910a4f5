"""CPU baseline leg of bench.py (TEST/MEASUREMENT INFRASTRUCTURE ONLY -- never the product path).

Times the REFERENCE CPU TNet (oracle/_ref/TNet: src/TNet.cc + TNetLib + KaldiLib compiled by
oracle/Makefile.ref, MKL standing in for the un-vendored GotoBLAS) on a bounded synthetic sample of
the benchmark workload, with the reference's own data-parallel Platform (--THREADS=T, bunch/T
rows per thread, src/TNetLib/Platform.h:143-391).

The reference's FPS line includes writing the trained model as text (src/TNet.cc:355-362), so the
compute-only rate is taken from two runs of different length: fps = d(frames) / d(seconds).
If the reference binary is absent the oracle restatement is timed instead (kind "port").
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_TNET = os.path.join(HERE, "_ref", "TNet")


def _zero_nnet_text(dims):
    """<biasedlinearity> weights as short "0" tokens (fast to write and parse; GEMM cost is
    value-independent) -- biases as in gen_mlp_init --negbias."""
    parts = []
    for i in range(len(dims) - 1):
        ni, no = dims[i], dims[i + 1]
        parts.append(f"<biasedlinearity> {no} {ni}\nm {no} {ni}\n")
        row = "0 " * ni + "\n"
        parts.append(row * no)
        bias = "0 " * no if i == len(dims) - 2 else "-4 " * no
        parts.append(f"v {no} {bias}\n")
        parts.append(f"<{'softmax' if i == len(dims) - 2 else 'sigmoid'}> {no} {no}\n")
    return "".join(parts)


def _write_corpus(outdir, n_frames, dim, n_cls, seed):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "nnet-asr_amd"))
    from tnet_amd import formats
    rng = np.random.default_rng(seed)
    lens, tot = [], 0
    while tot < n_frames:
        n = int(rng.integers(200, 1501))
        n = min(n, n_frames - tot) if n_frames - tot >= 200 else n
        lens.append(n)
        tot += n
    feats = [rng.standard_normal((n, dim)).astype(np.float32) for n in lens]
    labels = [rng.integers(0, n_cls, n).astype(np.int32) for n in lens]
    return formats.write_corpus_htk(formats.Corpus(feats, labels), outdir, n_cls)


def _run_tnet(files, init, outdir, bunch, cache, threads, lr=1e-4):
    env = dict(os.environ, MKL_NUM_THREADS="1", OMP_NUM_THREADS="1")
    cmd = [REF_TNET, "-H", init, "-I", files["mlf"], "-L", "*/", "-X", "lab", "-S", files["scp"], "-m",
           files["states"], "-n", repr(lr), f"--TARGETMMF={os.path.join(outdir, 'out.nnet')}",
           f"--BUNCHSIZE={bunch}", f"--CACHESIZE={cache}", "--RANDOMIZE=TRUE", "--SEED=123", f"--THREADS={threads}"]
    t0 = time.time()
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=outdir)
    wall = time.time() - t0
    if p.returncode != 0:
        raise RuntimeError(f"reference TNet failed: {p.stderr[-2000:]}")
    m = re.search(r"FINISHED \( ([0-9.e+]+)s \) \[ FPS: ([0-9.e+]+)", p.stdout)
    fr = re.search(r"frames:(\d+)", p.stdout)
    return float(m.group(1)), float(m.group(2)), int(fr.group(1)), wall


def reference_cpu_baseline(dims, bunch=1024, threads=None, bunches=(6, 22), seed=0):
    """Returns dict(value, unit, cores, kind, sample)."""
    if not os.path.exists(REF_TNET):
        return None
    threads = threads or min(16, os.cpu_count() or 1)
    # per-thread cache of 2048 rows (> the longest synthetic utterance, so no Platform abort;
    # Platform.h:159-160 derives it as (CACHESIZE/T/(B/T))*(B/T))
    cache = 2048 * threads
    tmp = tempfile.mkdtemp(prefix="tnet_cpu_")
    try:
        init = os.path.join(tmp, "init.nnet")
        import oracle as orc
        orc.write_random_nnet(init, dims, seed=2)
        # untimed warm-up run: pages MKL and the binary in from a cold image (on a fresh box the
        # first run is otherwise seconds slower, which corrupts the two-run slope)
        d = os.path.join(tmp, "warm")
        os.makedirs(d)
        files = _write_corpus(d, bunch + cache, dims[0], dims[-1], seed)
        _run_tnet(files, init, d, bunch, cache, threads)
        res = []
        for nb in bunches:
            d = os.path.join(tmp, f"run{nb}")
            os.makedirs(d)
            # enough frames for nb full global bunches even with per-thread cache tails
            files = _write_corpus(d, nb * bunch + cache, dims[0], dims[-1], seed)
            res.append(_run_tnet(files, init, d, bunch, cache, threads))
        (t1, fps1, f1, w1), (t2, fps2, f2, w2) = res
        if t2 <= t1 or f2 <= f1:
            raise RuntimeError(f"CPU baseline runs not monotone: {f1} frames {t1}s vs {f2} frames {t2}s")
        compute_fps = (f2 - f1) / (t2 - t1)
        return {"value": round(compute_fps, 1), "unit": "frames/s", "cores": threads, "kind": "reference",
                "sample": (f"reference TNet (src/TNet.cc, TNetLib Platform --THREADS={threads}, MKL 1 thread/worker) "
                           f"on synthetic {dims[0]}-dim frames, {'x'.join(map(str, dims))} net, bunch {bunch}: "
                           f"two runs of {f1} and {f2} trained frames, compute rate = dframes/dtime; "
                           f"reference-style FPS incl. model write {fps2:.1f}")}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def port_cpu_baseline(dims, bunch=1024, steps=2, seed=0):
    """The oracle restatement (fp64-accumulated C loops + OpenMP), used when _ref is absent."""
    import oracle as orc
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "nnet-asr_amd"))
    from tnet_amd import formats
    layers = formats.gen_mlp_init(dims, seed=2)
    net = orc.MLP.from_layers(layers)
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((bunch, dims[0])).astype(np.float32)
    L = rng.integers(0, dims[-1], bunch).astype(np.int32)
    t0 = time.time()
    for _ in range(steps):
        net.step(X, L, 1.0)
    dt = time.time() - t0
    return {"value": round(steps * bunch / dt, 1), "unit": "frames/s", "cores": os.cpu_count() or 1, "kind": "port",
            "sample": f"oracle restatement, {steps} SGD steps of {bunch} frames"}
