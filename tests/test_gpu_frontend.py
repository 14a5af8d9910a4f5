"""Feature front end on the GPU (--FEATURETRANSFORM networks, src/CuTNetLib/cuCRBEDctFeat.h:16-304):
every component through the C ABI vs the numpy restatement (oracle.frontend_component), the whole
Hamm_dct_norm-structured transform vs the reference CPU TFeaCat output (tests/golden/
frontend_feacat.npz), and the unmodified reference TNetCu / TFeaCatCu drivers with
--FEATURETRANSFORM on this library vs the reference CPU TNet / TFeaCat (make_frontend.py).

Tolerances: gathers / window / bias bit-exact; <blocklinearity> (fp32 fma chain vs float64) and
<log> rel 1e-5 / abs 1e-5; epoch Xent rel 1e-4, accuracy 0.05 % abs."""
import importlib.util
import json
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle as orc  # noqa: E402
import tnet_amd  # noqa: E402
from tnet_amd import formats  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mf():
    spec = importlib.util.spec_from_file_location("make_frontend", os.path.join(REPO, "tests", "golden",
                                                                                "make_frontend.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    return mf


def _forward(layers, x):
    net = tnet_amd.Network.from_layers(layers, precision=9)
    X = tnet_amd.DeviceArray.from_numpy(np.ascontiguousarray(x, np.float32))
    return net.propagate(X).numpy()


def _exact(L, x):
    np.testing.assert_array_equal(_forward([L], x), orc.frontend_component(L, x))


@pytest.mark.parametrize("rows", [1, 5, 333])
def test_expand(rows):
    rng = np.random.default_rng(rows)
    x = rng.standard_normal((rows, 23)).astype(np.float32)
    _exact(formats.Layer("<expand>", 23 * 5, 23, extra={"offsets": np.array([-4, -1, 0, 3, 9])}), x)


def test_copy_one_based_and_out_of_range():
    x = np.random.default_rng(1).standard_normal((40, 13)).astype(np.float32)
    idx = np.array([12, 0, 5, 5, 13, -7, 2])     # 13 and -7 are out of range -> +inf
    L = formats.Layer("<copy>", len(idx), 13, extra={"indices": idx})
    y = _forward([L], x)
    np.testing.assert_array_equal(y, orc.frontend_component(L, x))
    assert np.isinf(y[:, 4]).all() and np.isinf(y[:, 5]).all()


@pytest.mark.parametrize("ctx,ch", [(51, 23), (11, 3), (1, 7)])
def test_transpose(ctx, ch):
    x = np.random.default_rng(ctx).standard_normal((65, ctx * ch)).astype(np.float32)
    _exact(formats.Layer("<transpose>", ctx * ch, ctx * ch, extra={"context": ctx}), x)


def test_bias_window():
    rng = np.random.default_rng(4)
    x = rng.standard_normal((129, 598)).astype(np.float32)
    _exact(formats.Layer("<bias>", 598, 598, b=rng.standard_normal(598).astype(np.float32)), x)
    _exact(formats.Layer("<window>", 598, 598, extra={"window": rng.random(598).astype(np.float32)}), x)


def test_log():
    x = np.random.default_rng(5).random((77, 31)).astype(np.float32) * 10 + 1e-3
    L = formats.Layer("<log>", 31, 31)
    np.testing.assert_allclose(_forward([L], x), orc.frontend_component(L, x), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("bi,bo,nb,rows", [(51, 26, 23, 300), (7, 3, 5, 9), (1, 1, 4, 2), (200, 100, 2, 50),
                                           (64, 64, 3, 1)])
def test_blocklinearity(bi, bo, nb, rows):
    """Any block shape (odd offsets: the reference's per-block cublasSgemm has no alignment
    constraint either); 200x100 exceeds the LDS staging limit and reads the block from L2."""
    rng = np.random.default_rng(bi * 1000 + bo)
    B = rng.standard_normal((bi, bo)).astype(np.float32)
    L = formats.Layer("<blocklinearity>", nb * bo, nb * bi, W=B)
    x = rng.standard_normal((rows, nb * bi)).astype(np.float32)
    np.testing.assert_allclose(_forward([L], x), orc.frontend_component(L, x), rtol=1e-5, atol=1e-5)


def test_transform_vs_reference_tfeacat(golden_dir):
    """The whole transform on extended utterances vs the reference CPU TFeaCat output."""
    mf = _mf()
    corpus = formats.synth_corpus(**mf.CORPUS)
    layers = formats.round_trip_text(formats.gen_frontend_transform(**mf.TRANSFORM), 9)
    g = np.load(os.path.join(golden_dir, "frontend_feacat.npz"))
    net = tnet_amd.Network.from_layers(layers, precision=9)
    assert [c[0] for c in net.components()] == [L.tag for L in layers]
    for k, x in enumerate(corpus.feats):
        xe = formats.extend_frames(x, 25, 25)
        y = net.propagate(tnet_amd.DeviceArray.from_numpy(xe)).numpy()[25:-25]
        assert y.shape[0] == int(g["rows"][k])
        if k in mf.FULL:
            np.testing.assert_allclose(y, g[f"Y_{k}"], rtol=0, atol=2e-5)
        y = y.astype(np.float64)
        assert abs(y.sum() - g["sum"][k]) <= 1e-5 * np.abs(y).sum()
        assert abs((y ** 2).sum() - g["sumsq"][k]) <= 1e-5 * g["sumsq"][k]


def test_write_read_round_trip(tmp_path):
    layers = formats.gen_frontend_transform(dim=6, context=3, n_dct=4, seed=2) + [
        formats.Layer("<copy>", 5, 24, extra={"indices": np.array([0, 23, 4, 4, 1])}), formats.Layer("<log>", 5, 5)]
    net = tnet_amd.Network.from_layers(layers, precision=9)
    p = str(tmp_path / "t.nnet")
    net.write(p)
    back = formats.read_nnet(p)
    assert [(L.tag, L.n_out, L.n_in) for L in back] == [(L.tag, L.n_out, L.n_in) for L in layers]
    np.testing.assert_array_equal(back[0].extra["offsets"], layers[0].extra["offsets"])
    np.testing.assert_array_equal(back[6].extra["indices"], layers[6].extra["indices"])
    assert back[1].extra["context"] == 7
    np.testing.assert_allclose(back[3].W, layers[3].W, rtol=1e-5, atol=1e-6)   # 6 significant digits
    x = np.random.default_rng(0).random((20, 6)).astype(np.float32) + 0.5
    np.testing.assert_allclose(_forward(back, x), _forward(layers, x), rtol=1e-4, atol=1e-5)


def test_bad_files_and_backprop_errors():
    with pytest.raises(RuntimeError):       # offsets do not map 23 -> 100
        tnet_amd.Network(text="<expand> 100 23\nv 3  -1 0 1\n")
    with pytest.raises(RuntimeError):       # 10 not divisible by context 3
        tnet_amd.Network(text="<transpose> 10 10\n 3\n")
    with pytest.raises(RuntimeError):       # block 5x3 does not divide 12 -> 8
        tnet_amd.Network(text="<blocklinearity> 8 12\nm 3 5\n" + "1 " * 15 + "\n")
    net = tnet_amd.Network(text="<window> 4 4\nv 4  1 2 3 4\n")
    X = tnet_amd.DeviceArray.from_numpy(np.ones((3, 4), np.float32))
    net.propagate(X)
    with pytest.raises(RuntimeError):       # the reference: Error("__func__ Not implemented")
        net.backpropagate(X)
    b = tnet_amd.Network(text="<bias> 4 4\nv 4  1 2 3 4\n")
    b.propagate(X)
    b.backpropagate(X)                      # <bias> backpropagates a copy


# ------------------------------------------------------------------- reference drivers (drop-in)

def _driver(name):
    return os.path.join(REPO, "oracle", "_ref", f"{name}_amd")


@pytest.mark.skipif(not os.path.exists(_driver("TNetCu")), reason="oracle/_ref/TNetCu_amd not built")
def test_reference_tnetcu_with_featuretransform(golden_dir):
    """examples/01 run_test.GPU.sh recipe (bunch 960, cache 14400, --FEATURETRANSFORM, frame ext
    25) through the reference TNetCu on this library vs the reference CPU TNet (THREADS=1)."""
    mf = _mf()
    cfg = json.load(open(os.path.join(golden_dir, "frontend_epoch.json")))
    with tempfile.TemporaryDirectory() as td:
        _, files = mf.make_inputs(td)
        init = os.path.join(td, "init.nnet")
        formats.write_nnet(formats.gen_mlp_init(cfg["dims"], seed=cfg["init_seed"]), init, precision=6)
        p = subprocess.run([_driver("TNetCu"), "-H", init, "-I", files["mlf"], "-L", "*/", "-X", "lab", "-S",
                            files["scp"], "-m", files["states"], "-n", repr(cfg["lr"]),
                            f"--TARGETMMF={os.path.join(td, 'out.nnet')}", f"--BUNCHSIZE={cfg['bunch']}",
                            f"--CACHESIZE={cfg['cache']}", "--RANDOMIZE=TRUE", f"--SEED={cfg['seed']}",
                            "--GRADDIVFRM=FALSE", f"--FEATURETRANSFORM={files['transform']}",
                            f"--STARTFRMEXT={cfg['frm_ext']}", f"--ENDFRMEXT={cfg['frm_ext']}"],
                           capture_output=True, text=True, cwd=td, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    m = re.search(r"TR Xent:(\S+) frames:(\d+) err/frm:(\S+) correct\[(\S+)%\]", p.stdout)
    assert m, p.stdout[-2000:]
    assert int(m.group(2)) == cfg["frames"]
    assert abs(float(m.group(1)) - cfg["xent"]) <= 1e-4 * cfg["xent"]
    assert abs(float(m.group(4)) - cfg["correct_pct"]) <= 0.05


@pytest.mark.skipif(not os.path.exists(_driver("TFeaCatCu")), reason="oracle/_ref/TFeaCatCu_amd not built")
def test_reference_tfeacatcu_with_featuretransform(golden_dir):
    """decode.sh's TFeaCatCu call (transform + MLP + --GMMBYPASS) vs the reference CPU TFeaCat."""
    mf = _mf()
    g = np.load(os.path.join(golden_dir, "frontend_decode.npz"))
    with tempfile.TemporaryDirectory() as td:
        _, files = mf.make_inputs(td)
        init = os.path.join(td, "init.nnet")
        formats.write_nnet(formats.gen_mlp_init(mf.EPOCH["dims"], seed=mf.EPOCH["init_seed"]), init, precision=6)
        outdir = os.path.join(td, "out")
        os.makedirs(outdir)
        p = subprocess.run([_driver("TFeaCatCu"), "-S", files["scp"], "-H", init, "-l", outdir, "-y", "fea",
                            f"--FEATURETRANSFORM={files['transform']}", "--GMMBYPASS=TRUE", "--STARTFRMEXT=25",
                            "--ENDFRMEXT=25"], capture_output=True, text=True, cwd=td, timeout=600)
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
        for k, n in enumerate(files["names"]):
            y = formats.read_htk(os.path.join(outdir, n + ".fea")).astype(np.float64)
            assert y.shape[0] == int(g["rows"][k])
            if k == mf.DECODE:
                np.testing.assert_allclose(y, g[f"Y_{k}"], rtol=1e-4, atol=1e-4)
            assert abs(y.sum() - g["sum"][k]) <= 1e-4 * np.abs(y).sum()


def test_native_trainer_with_featuretransform(golden_dir):
    """The library's own TNetCu loop (tnet_trainer_*) with tnet_trainer_set_transform: same epoch
    as the reference CPU TNet with --FEATURETRANSFORM and frame extension 25 (frontend_epoch.json)."""
    mf = _mf()
    cfg = json.load(open(os.path.join(golden_dir, "frontend_epoch.json")))
    corpus = formats.synth_corpus(**mf.CORPUS)
    transform = tnet_amd.Network.from_layers(formats.gen_frontend_transform(**mf.TRANSFORM), precision=9)
    net = tnet_amd.Network.from_layers(formats.round_trip_text(formats.gen_mlp_init(cfg["dims"],
                                                                                    seed=cfg["init_seed"]), 6))
    net.set_learn_rate(cfg["lr"])
    net.set_grad_div_frm(False)
    obj = tnet_amd.Objective()
    tr = tnet_amd.Trainer(net, obj, bunchsize=cfg["bunch"], cachesize=cfg["cache"], seed=cfg["seed"])
    tr.set_transform(transform, cfg["frm_ext"], cfg["frm_ext"])
    tr.train_corpus(corpus.feats, corpus.labels)
    err, frames, correct = obj.stats()
    assert frames == cfg["frames"]
    np.testing.assert_allclose(err, cfg["xent"], rtol=1e-4)
    assert abs(100.0 * correct / frames - cfg["correct_pct"]) <= 0.05
