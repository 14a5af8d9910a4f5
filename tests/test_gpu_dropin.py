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
