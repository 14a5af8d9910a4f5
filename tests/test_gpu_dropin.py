"""Drop-in check: the reference's own TNetCu driver (src/TNetCu.cc, unmodified) and KaldiLib,
linked against this library instead of the CUDA CuBaseLib/CuTNetLib (oracle/Makefile.dropin ->
oracle/_ref/TNetCu_amd, built in the container from the reference sources; the binary travels to
the GPU box), trains one examples/01-style epoch with GRADDIVFRM=FALSE and must print the same
Report as the reference CPU TNet (THREADS=1) on the same files (tests/golden/epoch_mlp3*.json).
The GPU(GRADDIVFRM=F, momentum 0) == CPU(THREADS=1) equivalence is the reference's own
(tools/.../run_test.GPU.sh:50).  Tolerance: Xent relative 1e-4, accuracy 0.05 % absolute."""
import json
import os
import re
import subprocess
import tempfile

import pytest

pytestmark = pytest.mark.gpu

from tnet_amd import formats  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(REPO, "oracle", "_ref", "TNetCu_amd")


@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/TNetCu_amd not built (needs /root/reference)")
@pytest.mark.parametrize("name", ["epoch_mlp3.json", "epoch_mlp3_b256.json"])
def test_reference_tnetcu_driver_on_this_library(golden_dir, name):
    cfg = json.load(open(os.path.join(golden_dir, name)))
    corpus = formats.synth_corpus(cfg["n_utts"], cfg["dim"], cfg["n_cls"], seed=cfg["corpus_seed"],
                                  min_len=cfg["min_len"], max_len=cfg["max_len"])
    layers = formats.gen_mlp_init(cfg["dims"], seed=cfg["init_seed"])
    with tempfile.TemporaryDirectory() as td:
        files = formats.write_corpus_htk(corpus, td, cfg["n_cls"])
        init = os.path.join(td, "init.nnet")
        formats.write_nnet(layers, init, precision=6)
        out = os.path.join(td, "out.nnet")
        cmd = [DROPIN, "-H", init, "-I", files["mlf"], "-L", "*/", "-X", "lab", "-S", files["scp"], "-m",
               files["states"], "-n", repr(cfg["lr"]), f"--TARGETMMF={out}", f"--BUNCHSIZE={cfg['bunch']}",
               f"--CACHESIZE={cfg['cache']}", "--RANDOMIZE=TRUE", f"--SEED={cfg['seed']}", "--GRADDIVFRM=FALSE"]
        p = subprocess.run(cmd, capture_output=True, text=True, cwd=td, timeout=600)
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
        m = re.search(r"TR Xent:(\S+) frames:(\d+) err/frm:(\S+) correct\[(\S+)%\]", p.stdout)
        assert m, p.stdout[-2000:]
        assert int(m.group(2)) == cfg["frames"]
        assert abs(float(m.group(1)) - cfg["xent"]) <= 1e-4 * cfg["xent"]
        assert abs(float(m.group(4)) - cfg["correct_pct"]) <= 0.05
        # the written model is a valid .nnet of the same topology
        back = formats.read_nnet(out)
        assert [L.tag for L in back] == [L.tag for L in layers]


def _driver(name):
    return os.path.join(REPO, "oracle", "_ref", f"{name}_amd")


def _run(cmd, cwd):
    p = subprocess.run(cmd, capture_output=True, text=True, cwd=cwd, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    return p.stdout


@pytest.mark.skipif(not os.path.exists(_driver("TRbmCu")), reason="oracle/_ref/TRbmCu_amd not built")
def test_reference_trbmcu_driver_on_this_library():
    """TRbmCu (config 4's driver): Gauss-Bernoulli CD-1 epoch vs the oracle restatement (same lrand48
    stream: CuRand seeds first, then the cache shuffles).  Tolerances as tests/test_gpu_rbm.py, plus
    the 6-digit text of the written model."""
    import numpy as np
    import oracle as orc
    V, H, B, cache, seed, lr, mmt, wc = 40, 64, 32, 256, 321, 0.01, 0.5, 0.0002
    rng = np.random.default_rng(5)
    feats = [rng.standard_normal((int(n), V)).astype(np.float32) for n in rng.integers(40, 200, size=12)]
    layer = formats.round_trip_text(formats.gen_rbm_init(V, H, seed=6), 6)[0]
    with tempfile.TemporaryDirectory() as td:
        corpus = formats.Corpus(feats, [np.zeros(len(f), np.int32) for f in feats])
        files = formats.write_corpus_htk(corpus, td, 2)
        init = os.path.join(td, "rbm.nnet")
        formats.write_nnet([layer], init, precision=6)
        out = os.path.join(td, "out.nnet")
        txt = _run([_driver("TRbmCu"), "-H", init, "-S", files["scp"], "-n", repr(lr), f"--MOMENTUM={mmt}",
                    f"--WEIGHTCOST={wc}", f"--BUNCHSIZE={B}", f"--CACHESIZE={cache}", f"--SEED={seed}",
                    "--RANDOMIZE=TRUE", f"--TARGETMMF={out}"], td)
        back = formats.read_nnet(out)[0]
    rs = orc.RandState(seed, B, H)
    X = np.concatenate(feats)
    m = orc.RBM.from_layer(layer)
    for b in orc.epoch_schedule_x([len(f) for f in feats], cache, B, rs.x_after):
        m.step(X[b], rs, lr, mmt, wc)
    mm = re.search(r"Mse:(\S+) frames:(\d+)", txt)
    assert mm, txt[-2000:]
    assert int(mm.group(2)) == m.frames
    assert abs(float(mm.group(1)) - m.mse) <= 1e-4 * m.mse
    np.testing.assert_allclose(back.W, m.W, rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose(back.extra["vis_bias"], m.vb, rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose(back.b, m.hb, rtol=2e-4, atol=2e-5)


@pytest.mark.skipif(not os.path.exists(_driver("TRecurrentCu")), reason="oracle/_ref/TRecurrentCu_amd not built")
def test_reference_trecurrentcu_driver_on_this_library():
    """TRecurrentCu (config 5's driver): frame-by-frame BPTT epoch vs the oracle restatement."""
    import numpy as np
    import oracle as orc
    nIn, H, Sd, lr, bptt = 24, 32, 10, 0.05, 3
    rng = np.random.default_rng(9)
    feats = [rng.standard_normal((int(T), nIn)).astype(np.float32) for T in (50, 70, 30)]
    labels = [rng.integers(0, Sd, len(f)).astype(np.int32) for f in feats]
    layers = formats.round_trip_text(formats.gen_recurrent_init(nIn, H, Sd, seed=7), 6)
    with tempfile.TemporaryDirectory() as td:
        files = formats.write_corpus_htk(formats.Corpus(feats, labels), td, Sd)
        init = os.path.join(td, "rnn.nnet")
        formats.write_nnet(layers, init, precision=6)
        out = os.path.join(td, "out.nnet")
        txt = _run([_driver("TRecurrentCu"), "-H", init, "-I", files["mlf"], "-L", "*/", "-X", "lab", "-S",
                    files["scp"], "-m", files["states"], "-n", repr(lr), f"--BPTT={bptt}", f"--TARGETMMF={out}"], td)
    m = orc.RNN(layers[0].W, layers[0].b, layers[1].W, layers[1].b)
    for f, l in zip(feats, labels):
        m.utterance(f, l, bptt, lr)
    # TRecurrentCu prints "-- TR" + Report() without a space (TRecurrentCu.cc:410)
    mm = re.search(r"TR ?Xent:(\S+) frames:(\d+) err/frm:(\S+) correct\[(\S+)%\]", txt)
    assert mm, txt[-2000:]
    assert int(mm.group(2)) == m.frames
    assert abs(float(mm.group(1)) - m.xent) <= 1e-4 * m.xent
    assert abs(float(mm.group(4)) - 100.0 * m.correct / m.frames) <= 0.05


@pytest.mark.skipif(not os.path.exists(_driver("TFeaCatCu")), reason="oracle/_ref/TFeaCatCu_amd not built")
def test_reference_tfeacatcu_driver_on_this_library():
    """TFeaCatCu (forward-only driver): network outputs written as
    HTK features vs the oracle forward pass (rtol 1e-4)."""
    import numpy as np
    import oracle as orc
    dims = [30, 64, 64, 12]
    rng = np.random.default_rng(2)
    feats = [rng.standard_normal((int(T), dims[0])).astype(np.float32) for T in (20, 90)]
    layers = formats.round_trip_text(formats.gen_mlp_init(dims, seed=4), 6)
    with tempfile.TemporaryDirectory() as td:
        files = formats.write_corpus_htk(formats.Corpus(feats, [np.zeros(len(f), np.int32) for f in feats]), td, 2)
        init = os.path.join(td, "mlp.nnet")
        formats.write_nnet(layers, init, precision=6)
        outdir = os.path.join(td, "out")
        os.makedirs(outdir)
        _run([_driver("TFeaCatCu"), "-H", init, "-S", files["scp"], "-l", outdir, "-y", "fea"], td)
        names = [os.path.splitext(os.path.basename(l.strip()))[0] for l in open(files["scp"]) if l.strip()]
        outs = [formats.read_htk(os.path.join(outdir, n + ".fea")) for n in names]
    m = orc.MLP.from_layers(layers)
    for f, o in zip(feats, outs):
        np.testing.assert_allclose(o, m.forward(f), rtol=1e-4, atol=1e-6)
