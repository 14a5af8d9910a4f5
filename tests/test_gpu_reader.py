"""The TNetCu epoch fed by the native host front end (tnet_trainer_add_reader: FeatureReader ->
CuTrainer::AddUtteranceExtended, the cache fill of TNetCu.cc:376-419) on examples/01's own files.

Tolerance: none.  The reader delivers exactly the frames / class ids the reference's FeatureRepository /
LabelRepository do (tests/test_reader.py, bit-exact vs the reference), so an epoch fed by it must be
bit-identical to the same epoch fed from formats.read_corpus through add_utterance (whose Report
matches the reference CPU TNet's band, tests/test_ex01.py): same Xent / frames / correct, same weights."""
import json
import os

import numpy as np
import pytest

from tnet_amd import formats

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
EX = os.path.join(GOLD, "ex01")

pytestmark = pytest.mark.gpu


def _setup(cfg, init_cfg, transform_path):
    import tnet_amd
    transform = tnet_amd.Network(path=transform_path)
    net = tnet_amd.Network.from_layers(formats.round_trip_text(
        formats.gen_mlp_init(init_cfg["dims"], seed=init_cfg["seed"]), 6))
    net.set_learn_rate(cfg["lr"])
    net.set_grad_div_frm(False)
    obj = tnet_amd.Objective()
    tr = tnet_amd.Trainer(net, obj, bunchsize=cfg["bunch"], cachesize=cfg["cache"], seed=cfg["seed"])
    tr.set_transform(transform, cfg["frm_ext"], cfg["frm_ext"])
    return transform, net, obj, tr


@pytest.mark.parametrize("threads,depth", [(1, 1), (8, 16)])
def test_epoch_from_native_reader_equals_epoch_from_memory(threads, depth):
    import tnet_amd
    g = json.load(open(os.path.join(GOLD, "ex01_epoch.json")))
    init_cfg, cfg = g["init"], next(e for e in g["epochs"] if e["name"] == "run_test_cpu_b960")
    tpath = os.path.join(EX, "Hamm_dct_norm")

    c = formats.read_corpus(os.path.join(EX, "test.scp"), os.path.join(EX, "test_3s.mlf"),
                            os.path.join(EX, "mono_state_phn_set_135_phn"))
    keep_a = _setup(cfg, init_cfg, tpath)
    _, net_a, obj_a, tr_a = keep_a
    tr_a.train_corpus(c.feats, c.labels)

    keep_b = _setup(cfg, init_cfg, tpath)
    _, net_b, obj_b, tr_b = keep_b
    cwd = os.getcwd()
    os.chdir(EX)
    try:
        r = tnet_amd.FeatureReader("test.scp", mlf="test_3s.mlf", label_map="mono_state_phn_set_135_phn",
                                   start_ext=cfg["frm_ext"], end_ext=cfg["frm_ext"], threads=threads, depth=depth)
        added = tr_b.add_reader(r)
        tr_b.finish()
    finally:
        os.chdir(cwd)
    assert added == c.frames
    assert obj_a.stats()[1] == cfg["frames"]
    assert obj_b.stats() == obj_a.stats()
    assert tr_b.steps == tr_a.steps
    for (Wa, ba), (Wb, bb) in zip(net_a.linear_params(), net_b.linear_params()):
        assert np.array_equal(Wa, Wb) and np.array_equal(ba, bb)


def test_reader_extension_must_match_the_transform():
    """features carrying 10 context rows cannot feed a transform that expects 25 (an error, not a silent
    mis-trim)"""
    import tnet_amd
    g = json.load(open(os.path.join(GOLD, "ex01_epoch.json")))
    init_cfg, cfg = g["init"], next(e for e in g["epochs"] if e["name"] == "run_test_cpu_b960")
    keep = _setup(cfg, init_cfg, os.path.join(EX, "Hamm_dct_norm"))
    tr = keep[3]
    cwd = os.getcwd()
    os.chdir(EX)
    try:
        r = tnet_amd.FeatureReader("test.scp", mlf="test_3s.mlf", label_map="mono_state_phn_set_135_phn",
                                   start_ext=10, end_ext=10)
        with pytest.raises(tnet_amd.TnetError, match="the transform expects 25/25"):
            tr.add_reader(r, 1)
    finally:
        os.chdir(cwd)


def test_add_reader_rejects_invalid_values(tmp_path):
    """TNetCu checks every utterance for NaN / Inf before the transform (feats_host.CheckData,
    TNetCu.cc:386, Matrix.h:238-252): the reader's intake rejects it with the same message"""
    import tnet_amd
    os.makedirs(tmp_path / "f")
    x = np.zeros((20, 3), np.float32)
    x[7, 2] = np.nan
    formats.write_htk(str(tmp_path / "f" / "a.fea"), x)
    (tmp_path / "list.scp").write_text("f/a.fea\n")
    (tmp_path / "a.mlf").write_text('#!MLF!#\n"*/a.lab"\n0 2000000 s0\n.\n')
    (tmp_path / "states").write_text("s0\ns1\n")
    net = tnet_amd.Network.from_layers(formats.gen_mlp_init([3, 8, 2], seed=1))
    tr = tnet_amd.Trainer(net, tnet_amd.Objective(), bunchsize=4, cachesize=16, seed=1)
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        r = tnet_amd.FeatureReader("list.scp", mlf="a.mlf", label_map="states")
    finally:
        os.chdir(cwd)
    with pytest.raises(tnet_amd.TnetError, match=r"Invalid value: nan in matrix row: 7 col: 2 file: f/a.fea"):
        tr.add_reader(r)
