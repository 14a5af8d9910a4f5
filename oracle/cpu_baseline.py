"""CPU baseline leg of bench.py (TEST/MEASUREMENT INFRASTRUCTURE ONLY -- never the product path).

Times the REFERENCE CPU TNet (oracle/_ref/TNet: src/TNet.cc + TNetLib + KaldiLib compiled by
oracle/Makefile.ref, MKL standing in for the un-vendored GotoBLAS) on a bounded synthetic sample of
the benchmark workload, with the reference's own data-parallel Platform (--THREADS=T, bunch/T
rows per thread, src/TNetLib/Platform.h:143-391).

The reference's own FPS line includes reading and writing the model as text (src/TNet.cc:321-362),
which on the 16-CPU-quota GPU boxes swamps the training time; oracle/_ref/ref_harness `train`
therefore sets Platform up the way TNet.cc does and times RunTrain alone.  If the reference build
is absent the oracle restatement is timed instead (kind "port").
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


REF_HARNESS = os.path.join(HERE, "_ref", "ref_harness")


def cpu_quota():
    """CPUs this process may use: the cgroup v2 quota if one is set (the GPU boxes expose every
    host CPU to sched_getaffinity but cap the container at a 16-CPU quota), else the affinity."""
    n = len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def _run_platform(files, init, bunch, cache, threads, seed=123, lr=1e-4):
    """oracle/_ref/ref_harness train: the reference Platform::RunTrain, timed around the loop."""
    env = dict(os.environ, MKL_NUM_THREADS="1", OMP_NUM_THREADS="1")
    cmd = [REF_HARNESS, "train", init, files["scp"], files["mlf"], files["states"], "*/", str(threads), str(bunch),
           str(cache), repr(lr), str(seed)]
    p = subprocess.run(cmd, capture_output=True, text=True, env=env)
    m = re.search(r"HARNESS_RESULT frames (\d+) seconds ([0-9.e+-]+)", p.stderr)
    if not m:  # (a result line is complete: the timed loop had finished when it was printed)
        raise RuntimeError(f"reference Platform training failed (rc {p.returncode}): {p.stderr[-2000:]}")
    return int(m.group(1)), float(m.group(2))


def reference_cpu_baseline(dims, bunch=1024, threads=None, target_s=12.0, seed=0):
    """Returns dict(value, unit, cores, kind, sample)."""
    if not os.path.exists(REF_HARNESS):
        return None
    threads = threads or min(16, cpu_quota())
    # per-thread cache of 2048 rows (> the longest synthetic utterance, so no Platform abort;
    # Platform.h:159-160 derives it as (CACHESIZE/T/(B/T))*(B/T))
    cache = 2048 * threads
    tmp = tempfile.mkdtemp(prefix="tnet_cpu_")
    try:
        init = os.path.join(tmp, "init.nnet")
        import oracle as orc
        orc.write_random_nnet(init, dims, seed=2)
        # short run: pages MKL and the binary in, and sizes the timed sample
        d = os.path.join(tmp, "warm")
        os.makedirs(d)
        f0, t0 = _run_platform(_write_corpus(d, 4 * bunch + cache, dims[0], dims[-1], seed), init, bunch, cache,
                               threads)
        n_frames = int(min(max(f0 / max(t0, 1e-3) * target_s, 16 * bunch), 400_000))
        d = os.path.join(tmp, "timed")
        os.makedirs(d)
        frames, secs = _run_platform(_write_corpus(d, n_frames + cache, dims[0], dims[-1], seed + 1), init, bunch,
                                     cache, threads)
        return {"value": round(frames / secs, 1), "unit": "frames/s", "cores": threads, "kind": "reference",
                "sample": (f"reference TNet CPU training loop (TNetLib Platform::RunTrain, Platform.h:143-198, "
                           f"{threads} SGD threads + reader, MKL 1 thread/worker standing in for GotoBLAS) compiled "
                           f"from the reference sources (oracle/Makefile.ref), {'x'.join(map(str, dims))} net, "
                           f"bunch {bunch}, synthetic {dims[0]}-dim HTK features: {frames} frames in {secs:.2f} s "
                           f"timed around RunTrain (model read/write excluded)")}
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
