#!/usr/bin/env python3
"""Host front end throughput ("at ~1 M frames/s/GPU the host front end
becomes the bottleneck"): HTK feature files + MLF read by the native reader (csrc/host/htkio.cpp) against
the rate the GPU trainer consumes them.

Corpus: synthetic 440-dim big-endian HTK USER files (the metric network's input; lengths uniform in
[200, 1500] frames), state runs of 3..12 frames in an MLF over 4000 states, written to a
scratch directory first (so the reads below come from the page cache: decode + copy, not the disk).

  reader   : frames/s of FeatureReader alone (features + class ids, no copies out), per thread count
  train    : Trainer.add_reader over the same files on the dnn4 network (440:2048x4:4000, bunch 1024,
             cache 16384, GRADDIVFRM): the TNetCu epoch loop read from disk, trained on the GPU
  memory   : the same utterances handed to Trainer.add_utterance from numpy memory (tools/intake_bench.py)

usage: python tools/reader_bench.py [frames] [outdir]   (prints one JSON line)"""
import json
import os
import shutil
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
import numpy as np  # noqa: E402

from tnet_amd import FeatureReader, formats  # noqa: E402


def write_corpus(td, frames, dim, n_states, seed=0):
    rng = np.random.default_rng(seed)
    lens = []
    while sum(lens) < frames:
        lens.append(int(rng.integers(200, 1501)))
    os.makedirs(os.path.join(td, "feats"), exist_ok=True)
    scp, mlf = [], ["#!MLF!#"]
    for i, n in enumerate(lens):
        name = f"u{i:05d}"
        formats.write_htk(os.path.join(td, "feats", name + ".fea"), rng.standard_normal((n, dim), dtype=np.float32))
        scp.append(f"feats/{name}.fea")
        mlf.append(f'"*/{name}.lab"')
        t = 0
        while t < n:
            e = min(n, t + int(rng.integers(3, 13)))
            mlf.append(f"{t * 100000} {e * 100000} s{int(rng.integers(0, n_states))}")
            t = e
        mlf.append(".")
    open(os.path.join(td, "train.scp"), "w").write("\n".join(scp) + "\n")
    open(os.path.join(td, "train.mlf"), "w").write("\n".join(mlf) + "\n")
    open(os.path.join(td, "states"), "w").write("\n".join(f"s{i}" for i in range(n_states)) + "\n")
    return sum(lens), len(lens)


def reader_rate(td, threads, depth=32):
    cwd = os.getcwd()
    os.chdir(td)  # script paths are relative to the working directory, as the reference's
    try:
        t0 = time.perf_counter()
        r = FeatureReader("train.scp", mlf="train.mlf", label_map="states", threads=threads, depth=depth)
        n = 0
        while True:
            u = r.next_raw()
            if u is None:
                break
            n += u[1].shape[0]
        return n, time.perf_counter() - t0
    finally:
        os.chdir(cwd)


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 400000
    dims = [440, 2048, 2048, 2048, 2048, 4000]
    td = tempfile.mkdtemp(prefix="tnet_reader_", dir=os.environ.get("TMPDIR", "/tmp"))
    out = {"what": "native HTK/MLF reader (csrc/host/htkio.cpp) vs the GPU trainer's consumption",
           "dim": dims[0], "page_cache": "warm (files written just before; decode + copy, not disk)"}
    try:
        t0 = time.perf_counter()
        total, n_utts = write_corpus(td, frames, dims[0], dims[-1])
        out.update(frames=total, utterances=n_utts, bytes=total * dims[0] * 4 + 12 * n_utts,
                   write_s=round(time.perf_counter() - t0, 2))
        reader_rate(td, 8)  # warm the page cache
        rates = {}
        for th in (1, 2, 4, 8, 16):
            n, dt = reader_rate(td, th)
            assert n == total
            rates[str(th)] = {"frames_per_s": round(n / dt), "GB_per_s": round(n * dims[0] * 4 / dt / 1e9, 2)}
            print(f"reader threads {th}: {n / dt:.0f} frames/s", file=sys.stderr, flush=True)
        out["reader"] = rates
        if "--no-gpu" not in sys.argv:
            import bench
            import tnet_amd
            from tnet_amd import Objective, Trainer

            def trainer():
                net = bench.build_network(dims)
                net.set_learn_rate(1.0)
                net.set_grad_div_frm(True)
                return Trainer(net, Objective(), bunchsize=1024, cachesize=16384, seed=123, randomize=True), net

            # warm-up: allocations and code objects on a short list
            tr, _ = trainer()
            cwd = os.getcwd()
            os.chdir(td)
            try:
                r = FeatureReader("train.scp", mlf="train.mlf", label_map="states", threads=8, depth=32)
                tr.add_reader(r, 20)
                tr.finish()
                tnet_amd.synchronize()
                tr, _ = trainer()
                r = FeatureReader("train.scp", mlf="train.mlf", label_map="states", threads=8, depth=32)
                tnet_amd.synchronize()
                t0 = time.perf_counter()
                added = tr.add_reader(r)
                tr.finish()
                tnet_amd.synchronize()
                dt = time.perf_counter() - t0
            finally:
                os.chdir(cwd)
            out["train_from_files"] = {"frames_added": added, "frames_trained": tr.steps * 1024,
                                       "seconds": round(dt, 3), "frames_per_s": round(tr.steps * 1024 / dt),
                                       "reader_threads": 8}
            # the same utterances from numpy memory
            os.chdir(td)
            try:
                utts = [(x.copy(), lab.copy()) for _, x, lab, _, _ in
                        FeatureReader("train.scp", mlf="train.mlf", label_map="states", threads=8)]
            finally:
                os.chdir(cwd)
            tr, _ = trainer()
            tnet_amd.synchronize()
            t0 = time.perf_counter()
            for x, lab in utts:
                tr.add_utterance(x, lab)
            tr.finish()
            tnet_amd.synchronize()
            dt = time.perf_counter() - t0
            out["train_from_memory"] = {"frames_trained": tr.steps * 1024, "seconds": round(dt, 3),
                                        "frames_per_s": round(tr.steps * 1024 / dt)}
    finally:
        shutil.rmtree(td, ignore_errors=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
