"""Native host front end (csrc/host/htkio.cpp; include/tnet_train.h tnet_reader_*, tnet_htk_read) against
the reference's own FeatureRepository / LabelRepository (src/KaldiLib/Features.cc:1009-1347,
Labels.cc:42-186), run here through oracle/_ref/ref_harness `features` (tests/golden/make_reader.py ->
tests/golden/reader.npz: the synthetic HTK inputs are stored in the fixture, examples/01's are
tests/golden/ex01).

Tolerance: none -- features, class ids, shapes, sample periods and parameter kinds are bit-exact (the
reader only moves, byte-swaps and int16-decodes values; the _Z mean and the delta / acceleration
columns use the reference's float operation order).  Error records: the native message equals the
reference's exception text (KaldiLib's "(function:file:line)" prefix and stack trace removed); for the
unlabelled-frame error the reference also prints the all-zero one-hot row, compared up to it.

Pure host code: runs on CPU (no device calls)."""
import hashlib
import json
import os

import numpy as np
import pytest

from tnet_amd import FeatureReader, TnetError, formats, htk_read

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
EX = os.path.join(GOLD, "ex01")

_G = np.load(os.path.join(GOLD, "reader.npz"))
META = json.loads(bytes(_G["meta"]).decode())


@pytest.fixture(scope="module")
def workdir(tmp_path_factory):
    td = tmp_path_factory.mktemp("reader")
    os.makedirs(td / "d")
    for n in META["files"]:
        (td / "d" / n).write_bytes(bytes(_G[f"file:{n}"]))
    (td / "fb.fea").write_bytes(bytes(_G["file:fb.fea"]))
    (td / "test.mlf").write_bytes(bytes(_G["mlf"]))
    (td / "states.txt").write_bytes(bytes(_G["states"]))
    for k in _G.files:  # per-config MLFs (make_reader.py lookup_mlf: LabelContainer's lookup order)
        if k.startswith("mlf:"):
            (td / k[4:]).write_bytes(bytes(_G[k]))
        if k.startswith("norm:"):  # CMEANDIR / VARSCALEDIR / VARSCALEFN files (make_reader.py norm_files)
            os.makedirs(td / os.path.dirname(k[5:]), exist_ok=True)
            (td / k[5:]).write_bytes(bytes(_G[k]))
    return td


def _kind(name):
    """TARGETKIND text -> HTK kind code (FeatureRepository::ReadParmKind) and DERIVWINDOWS-less order"""
    base = {"ANON": 12, "MFCC": 6, "FBANK": 7, "USER": 9}
    parts = name.split("_")
    k = base[parts[0]]
    q = {"E": 0o100, "N": 0o200, "D": 0o400, "A": 0o1000, "Z": 0o4000, "0": 0o20000, "T": 0o100000}
    for p in parts[1:]:
        k |= q[p]
    order = 3 if k & 0o100000 else 2 if k & 0o1000 else 1 if k & 0o400 else 0
    return k, order


def _reader(td, name, threads=3, depth=2):
    c = META["configs"][name]
    scp = td / f"{name}.scp"
    scp.write_text("\n".join(c["scp"]) + "\n")
    kind, order = _kind(c["target_kind"])
    cwd = os.getcwd()
    os.chdir(td)
    try:
        mlf = c["mlf"] if isinstance(c["mlf"], str) else ("test.mlf" if c["mlf"] else None)
        norm = c.get("norm") or [None] * 5
        return FeatureReader(str(scp), mlf=mlf, label_map="states.txt", cmn_dir=norm[0], cmn_mask=norm[1],
                             cvn_dir=norm[2], cvn_mask=norm[3], cvg_file=norm[4],
                             label_dir=c["label_dir"], start_ext=c["start_ext"], end_ext=c["end_ext"],
                             swap=bool(c["swap"]), target_kind=kind, deriv_order=order, threads=threads, depth=depth)
    finally:
        os.chdir(cwd)


OK_CONFIGS = [n for n, c in META["configs"].items() if all("error" not in r for r in c["records"])]
ERR_CONFIGS = [n for n, c in META["configs"].items() if any("error" in r for r in c["records"])]


@pytest.mark.parametrize("name", OK_CONFIGS)
def test_reader_matches_reference_feature_repository(workdir, name):
    cwd = os.getcwd()
    r = _reader(workdir, name)
    os.chdir(workdir)
    try:
        got = list(r)
    finally:
        os.chdir(cwd)
    recs = META["configs"][name]["records"]
    assert len(got) == len(recs)
    for k, (rec, (logical, x, lab, per, kind)) in enumerate(zip(recs, got)):
        ref_x, ref_lab = _G[f"{name}:x{k}"], _G[f"{name}:lab{k}"]
        assert (x.shape, per, kind, logical) == ((rec["rows"], rec["cols"]), rec["period"], rec["kind"], rec["logical"])
        assert np.array_equal(x.view(np.uint32), ref_x.view(np.uint32)), f"{name} record {k}: features differ"
        lab = np.zeros(0, np.int32) if lab is None else lab  # no MLF: the reference writes no class ids
        assert np.array_equal(lab, ref_lab), f"{name} record {k}: class ids differ"


@pytest.mark.parametrize("name", ERR_CONFIGS)
def test_reader_errors_match_reference(workdir, name):
    ref = META["configs"][name]["records"][0]["error"]
    cwd = os.getcwd()
    r = _reader(workdir, name)
    os.chdir(workdir)
    try:
        with pytest.raises(TnetError) as ei:
            list(r)
    finally:
        os.chdir(cwd)
    native = str(ei.value).split("reader_next: status ", 1)[1].split(": ", 1)[1].strip()
    want = ref.split(" content:")[0].strip()
    assert native.startswith(want), (native, want)


def test_reader_examples01_matches_reference():
    """the first 20 examples/01 utterances with the run_test recipe's 25 / 25 frame extension and the MLF:
    float bytes (sha256), shapes and class ids as the reference's FeatureRepository / LabelRepository"""
    ex = META["ex01"]
    cwd = os.getcwd()
    os.chdir(EX)
    try:
        lines = [l.strip() for l in open("test.scp") if l.strip()][:20]
        r = FeatureReader("test.scp", mlf="test_3s.mlf", label_map="mono_state_phn_set_135_phn", start_ext=25,
                          end_ext=25, threads=4, depth=8)
        for k, rec in enumerate(ex["records"]):
            logical, x, lab, per, kind = r.next_raw()
            assert logical == lines[k] == rec["utt"]
            assert (x.shape, per, kind) == ((rec["rows"], rec["cols"]), rec["period"], rec["kind"])
            assert hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest() == rec["sha256"]
            assert np.array_equal(lab, _G[f"ex01:lab{k}"])
    finally:
        os.chdir(cwd)


def test_reader_matches_python_reader_on_all_of_examples01():
    """all 100 utterances, native vs tnet_amd.formats (itself pinned by the reference epoch fixtures)"""
    c = formats.read_corpus(os.path.join(EX, "test.scp"), os.path.join(EX, "test_3s.mlf"),
                            os.path.join(EX, "mono_state_phn_set_135_phn"))
    cwd = os.getcwd()
    os.chdir(EX)
    try:
        got = list(FeatureReader("test.scp", mlf="test_3s.mlf", label_map="mono_state_phn_set_135_phn", threads=8,
                                 depth=4))
    finally:
        os.chdir(cwd)
    assert len(got) == 100
    for (_, x, lab, per, _), xr, lr in zip(got, c.feats, c.labels):
        assert np.array_equal(x, xr) and np.array_equal(lab, lr) and per == 100000


@pytest.mark.parametrize("threads,depth", [(1, 1), (2, 1), (8, 3), (16, 64)])
def test_reader_order_and_rewind(threads, depth):
    """script order whatever the pool size / read-ahead depth; rewind restarts the list"""
    cwd = os.getcwd()
    os.chdir(EX)
    try:
        r = FeatureReader("test.scp", mlf="test_3s.mlf", label_map="mono_state_phn_set_135_phn", threads=threads,
                          depth=depth)
        assert len(r) == 100
        first = [(n, x.sum(dtype=np.float64)) for n, x, *_ in r]
        assert [n for n, _ in first] == [l.strip() for l in open("test.scp") if l.strip()]
        r.rewind()
        again = [(n, x.sum(dtype=np.float64)) for n, x, *_ in r]
        assert again == first
    finally:
        os.chdir(cwd)


def test_htk_read_single_record(workdir):
    """tnet_htk_read: one record without a reader, incl. a [s,e] range and edge extension"""
    x, per, kind = htk_read(str(workdir / "d" / "long.fea") + "[5,20]", start_ext=3, end_ext=3)
    assert np.array_equal(x, _G["ranges:x0"]) and per == 100000 and kind == 7
    full = formats.read_htk(str(workdir / "d" / "long.fea"))
    y, _, _ = htk_read(str(workdir / "d" / "long.fea"), start_ext=2, end_ext=4)
    assert np.array_equal(y, formats.extend_frames(full, 2, 4))


def test_reader_missing_script():
    with pytest.raises(TnetError, match="Cannot not open list file"):
        FeatureReader("/nonexistent/list.scp")


def test_reader_paths_fixed_at_creation(tmp_path):
    """relative script paths resolve against the working directory at creation: the pool reads ahead, so a
    later chdir (the consumer's business) must not move them"""
    cwd = os.getcwd()
    os.chdir(EX)
    try:
        r = FeatureReader("test.scp", mlf="test_3s.mlf", label_map="mono_state_phn_set_135_phn", threads=2, depth=2)
    finally:
        os.chdir(cwd)
    os.chdir(tmp_path)
    try:
        n = sum(1 for _ in r)
    finally:
        os.chdir(cwd)
    assert n == 100


def test_reader_under_sanitizers():
    """tools/htkio_sanitize.sh: the reader built with ThreadSanitizer (the read-ahead pool: several pool
    shapes, rewind mid-list, a reader abandoned with workers still reading) and with AddressSanitizer +
    UndefinedBehaviorSanitizer (the decoders) over examples/01, with and without frame extension"""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("no host compiler")
    p = subprocess.run([os.path.join(REPO, "tools", "htkio_sanitize.sh")], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert p.stdout.count("htkio_sanitize ok") == 4


def test_reader_norm_paths_fixed_at_creation(workdir, tmp_path):
    """relative CMEANDIR / VARSCALEDIR / VARSCALEFN resolve against the working directory at creation too: the
    pool reads ahead (and opens the normalisation files) after the constructor returns, so a chdir right after it
    must not move them (the reference opens them later from the same directory); error texts keep the names as
    given (test_reader_errors_match_reference)"""
    names = [n for n in OK_CONFIGS if META["configs"][n].get("norm")]
    assert names
    for name in names:
        for _ in range(3):
            r = _reader(workdir, name, threads=4, depth=4)  # returns with the cwd already restored
            cwd = os.getcwd()
            os.chdir(tmp_path)
            try:
                got = list(r)
            finally:
                os.chdir(cwd)
            assert len(got) == len(META["configs"][name]["records"])
