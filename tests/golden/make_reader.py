"""Golden vectors for the native host front end (csrc/host/htkio.cpp, tnet_reader_*): the reference's own
FeatureRepository / LabelRepository (src/KaldiLib/Features.cc, Labels.cc, built here by oracle/Makefile.ref)
run through oracle/_ref/ref_harness `features` over

  ex01  : the first 20 utterances of examples/01 (tests/golden/ex01), STARTFRMEXT / ENDFRMEXT 25, the MLF
  kinds : synthetic HTK files covering the parameter-kind logic -- plain FBANK, compressed FBANK_C,
          MFCC_E_D_A read as ANON (derivatives dropped), MFCC_E -> MFCC_E_D_A (deltas computed),
          MFCC_0 -> MFCC_Z (C0 dropped, sentence mean), logical=physical[s,e] frame ranges with context
          taken from real neighbours, NATURALREADORDER (little-endian data, no swap), MLF patterns
          ("*/x.lab", an exact name, a glob) and failing records (missing file, unknown state tag, a frame
          labelled twice, an unlabelled frame, no MLF record, an impossible TARGETKIND) and a range past
          the end of the file (edge-padded by the reference)

Writes tests/golden/reader.npz: the synthetic input files (bytes), scripts, MLF and state map, and per
configuration the reference's index (rows, cols, period, kind, error text) with the matrices (small
cases in full, ex01 as sha256 of the float32 bytes) and class ids.  Run in the build container
(needs /root/reference and `make -C oracle ref`); the test never needs the reference.
"""
import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
EX = os.path.join(HERE, "ex01")

FBANK, MFCC = 7, 6
E, N, D, A, C, Z, K0 = 0o100, 0o200, 0o400, 0o1000, 0o2000, 0o4000, 0o20000


def htk_bytes(x, period, kind, little=False):
    x = np.asarray(x, np.float32)
    n, d = x.shape
    e = "<" if little else ">"
    return struct.pack(e + "iihH", n, period, d * 4, kind) + x.astype(e + "f4").tobytes()


def htk_compressed_bytes(x, period, kind):
    """HTK compressed form: header (nSamples counts the 4 extra int16 'frames' of the scale / bias
    vectors), scale A and bias B as float32, then int16 frames: x = (s + B) / A"""
    x = np.asarray(x, np.float32)
    n, d = x.shape
    xmax, xmin = x.max(0), x.min(0)
    A = (2 * 32767.0 / np.maximum(xmax - xmin, 1e-3)).astype(np.float32)
    B = ((xmax + xmin) * A / 2).astype(np.float32)
    s = np.clip(np.round(x * A - B), -32767, 32767).astype(">i2")
    return (struct.pack(">iihH", n + 4, period, d * 2, kind | C) + A.astype(">f4").tobytes() + B.astype(">f4").tobytes()
            + s.tobytes())


def synthetic(rng):
    files, mlf, P = {}, ["#!MLF!#"], 100000

    def lab(name, n, segs=None, pattern=None):
        mlf.append(f'"{pattern or "*/" + name + ".lab"}"')
        if segs is None:  # runs of 1..7 frames over states s0..s9
            t, segs = 0, []
            while t < n:
                L = int(rng.integers(1, 8))
                segs.append((t, min(n, t + L), f"s{int(rng.integers(0, 10))}"))
                t += L
        for b, e, tag in segs:
            mlf.append(f"{b * P} {e * P} {tag}")
        mlf.append(".")

    x = rng.standard_normal((40, 12)).astype(np.float32)
    files["fb.fea"] = htk_bytes(x, P, FBANK)
    lab("fb", 40)
    files["fbc.fea"] = htk_compressed_bytes(rng.standard_normal((33, 10)) * 3, P, FBANK)
    lab("fbc", 33)
    files["mfeda.fea"] = htk_bytes(rng.standard_normal((25, 39)), P, MFCC | E | D | A)
    lab("mfeda", 25)
    files["mfe.fea"] = htk_bytes(rng.standard_normal((30, 13)), P, MFCC | E)
    lab("mfe", 30)
    files["mf0.fea"] = htk_bytes(rng.standard_normal((28, 13)) + 2.0, P, MFCC | K0)
    lab("mf0", 28)
    files["long.fea"] = htk_bytes(rng.standard_normal((60, 8)), P, FBANK)
    lab("long", 60)
    files["le.fea"] = htk_bytes(rng.standard_normal((20, 6)), P, FBANK, little=True)
    lab("le", 20)
    # label-side cases, all over long.fea's frames via logical names
    lab("exact", 60, pattern="lab/exact.lab")
    lab("globbed", 60, pattern="*/glob?.lab")
    lab("unk", 60, segs=[(0, 30, "s1"), (30, 60, "nosuchstate")])
    lab("twice", 60, segs=[(0, 31, "s1"), (30, 60, "s2")])
    lab("gap", 60, segs=[(0, 29, "s1"), (30, 60, "s2")])
    lab("trunc", 60, segs=[(0, 50, "s1"), (50, 80, "s3")])
    # the ranged records' labels: logical names r1..r3
    lab("r1", 16)
    lab("r2", 11)
    lab("r3", 20)
    lab("r9", 21)
    states = "\n".join(f"s{i}" for i in range(10)) + "\n"
    return files, "\n".join(mlf) + "\n", states


def lookup_mlf():
    """LabelContainer's lookup order (MlfStream.cc:43-265): every record labels all 60 frames of
    long.fea with its own state, so the class ids show which record a label resolved to.
      a: a later exact pattern that an earlier list pattern already matches is never hashed (the list wins)
      b: a hashed pattern resolves before a list pattern defined AFTER it
      c: a hash hit is overridden by a list pattern defined BEFORE it that matches the label (not the pattern)
      d: '*d1.lab' (no '/') is hashed at depth 0: it matches the label 'd1.lab' only (x/d1 has no record)
      e: a plain name defined after a list pattern that matches it is never hashed
      f: a label with a leading '/' and fewer '/' than a recorded depth: FindInHash's backward search wraps
         (find_last_of from prev - 1 at prev 0) and lands on the depth-1 key before the depth-2 one
      g/h: [..] and [!..] sets in list patterns"""
    mlf = ["#!MLF!#"]

    def rec(pattern, state):
        mlf.extend([f'"{pattern}"', f"0 {60 * 100000} s{state}", "."])
    rec("*/a?.lab", 1)
    rec("*/a1.lab", 2)
    rec("*/b1.lab", 3)
    rec("*/b?.lab", 4)
    rec("x/c?.lab", 5)
    rec("*/c1.lab", 6)
    rec("*d1.lab", 7)
    rec("*/e?.lab", 8)
    rec("x/e1.lab", 9)
    rec("*/p/q/r.lab", 0)
    rec("*/y/f1.lab", 2)
    rec("*/f1.lab", 3)
    rec("*/g[0-3]?.lab", 4)
    rec("*/h[!0-3]?.lab", 5)
    return "\n".join(mlf) + "\n"


def norm_files(rng):
    """cepstral mean / variance files for the CMEANDIR / VARSCALEDIR / VARSCALEFN cases (Features.cc:96-178,
    1352-1410): per-speaker files named by the first four characters of the logical name (mask %%%%*)"""
    f = {}

    def vec(n, lo=-1.0, hi=1.0):
        return " ".join(f"{v:.7g}" for v in rng.uniform(lo, hi, n))
    for spk in ("spkA", "spkB"):
        f[f"norm/cmn/{spk}"] = f"<CEPSNORM> <FBANK>\n<MEAN> 12\n{vec(12)}\n"
        f[f"norm/cvn/{spk}"] = f"<CEPSNORM> <FBANK>\n<VARIANCE> 12\n{vec(12, 0.2, 4.0)}\n"
        f[f"norm/cmn_eda/{spk}"] = f"<cepsnorm> <MFCC_E>\n<mean> 13\n{vec(13)}\n"
        f[f"norm/cvn_eda/{spk}"] = f"<CEPSNORM> <MFCC_E_D_A>\n<VARIANCE> 39\n{vec(39, 0.2, 4.0)}\n"
        f[f"norm/cmn_z/{spk}"] = f"<CEPSNORM> <MFCC_0>\n<MEAN> 13\n{vec(13)}\n"
    f["norm/varscale12"] = f"<VARSCALE> 12\n{vec(12, 0.5, 2.0)}\n"
    f["norm/bad/kind/spkA"] = f"<CEPSNORM> <MFCC>\n<MEAN> 12\n{vec(12)}\n"
    f["norm/bad/count/spkA"] = f"<CEPSNORM> <FBANK>\n<MEAN> 11\n{vec(11)}\n"
    f["norm/bad/eof/spkA"] = f"<CEPSNORM> <FBANK>\n<MEAN> 12\n{vec(7)}\n"
    f["norm/bad/junk/spkA"] = f"<CEPSNORM> <FBANK>\n<MEAN> 12\n{vec(12)} extra\n"
    f["norm/bad/word/spkA"] = f"<CEPSNORM> <FBANK>\n<MEAN> 12\n{vec(5)} x7 {vec(6)}\n"
    return f


SPK = ["spkA_u1=d/fb.fea", "spkB_u2=d/fb.fea", "spkA_u3=d/fb.fea"]

CONFIGS = {
    # name: (scp lines, swap, sext, eext, TARGETKIND, mlf?, label_dir)
    "plain": (["d/fb.fea", "d/fbc.fea", "d/long.fea"], 1, 3, 2, "ANON", True, None),
    "mfeda_anon": (["d/mfeda.fea"], 1, 0, 0, "ANON", True, None),
    "mfe_to_eda": (["d/mfe.fea"], 1, 2, 2, "MFCC_E_D_A", True, None),
    "mf0_to_z": (["d/mf0.fea"], 1, 0, 0, "MFCC_Z", True, None),
    "ranges": (["x/r1=d/long.fea[5,20]", "x/r2=d/long.fea[0,10]", "x/r3=d/long.fea[40,59]"], 1, 3, 3, "ANON", True,
               None),
    "natural": (["d/le.fea"], 0, 1, 1, "ANON", True, None),
    "patterns": (["exact=d/long.fea", "glob7=d/long.fea", "trunc=d/long.fea"], 1, 0, 0, "ANON", True, "lab"),
    "past_end": (["x/r9=d/long.fea[50,70]"], 1, 2, 2, "ANON", True, None),
    # failing records, one script each (after a GenDesiredMatrix exception the reference's MLF stream
    # stays open and its next lookup fails: the intake stops at the first error anyway)
    "err_missing": (["d/missing.fea"], 1, 0, 0, "ANON", True, None),
    "err_unknown_tag": (["x/unk=d/long.fea"], 1, 0, 0, "ANON", True, None),
    "err_twice": (["x/twice=d/long.fea"], 1, 0, 0, "ANON", True, None),
    "err_gap": (["x/gap=d/long.fea"], 1, 0, 0, "ANON", True, None),
    "err_no_record": (["fb.fea"], 1, 0, 0, "ANON", True, None),
    "err_convert": (["d/fb.fea"], 1, 0, 0, "MFCC", True, None),
    # LabelContainer lookup order (lookup_mlf)
    "mlf_lookup": (["x/a1=d/long.fea", "x/b1=d/long.fea", "x/c1=d/long.fea", "d1=d/long.fea", "x/e1=d/long.fea",
                    "/y/f1=d/long.fea", "x/g2z=d/long.fea", "x/h7z=d/long.fea"], 1, 0, 0, "ANON", "lookup.mlf", None),
    "err_mlf_depth0": (["x/d1=d/long.fea"], 1, 0, 0, "ANON", "lookup.mlf", None),
    "err_mlf_set": (["x/h2z=d/long.fea"], 1, 0, 0, "ANON", "lookup.mlf", None),
    # CMEANDIR / VARSCALEDIR / VARSCALEFN (8th field: cmn dir, cmn mask, cvn dir, cvn mask, VARSCALEFN)
    "norm_cmn": (SPK, 1, 2, 1, "ANON", False, None, ("norm/cmn", "%%%%*", None, None, None)),
    "norm_all": (SPK, 1, 2, 1, "ANON", False, None, ("norm/cmn", "%%%%*", "norm/cvn", "%%%%*", "norm/varscale12")),
    "norm_eda": (["spkA_e=d/mfe.fea", "spkB_e=d/mfe.fea"], 1, 2, 2, "MFCC_E_D_A", False, None,
                 ("norm/cmn_eda", "%%%%*", "norm/cvn_eda", "%%%%*", None)),
    "norm_z": (["spkB_z=d/mf0.fea"], 1, 0, 0, "MFCC_0_Z", False, None, ("norm/cmn_z", "%%%%*", None, None, None)),
    "err_norm_nomatch": (["u1=d/fb.fea"], 1, 0, 0, "ANON", False, None, ("norm/cmn", "%%%%?*", None, None, None)),
    "err_norm_kind": (["spkA_u1=d/fb.fea"], 1, 0, 0, "ANON", False, None, ("norm/bad/kind", "%%%%*", None, None, None)),
    "err_norm_count": (["spkA_u1=d/fb.fea"], 1, 0, 0, "ANON", False, None,
                       ("norm/bad/count", "%%%%*", None, None, None)),
    "err_norm_eof": (["spkA_u1=d/fb.fea"], 1, 0, 0, "ANON", False, None, ("norm/bad/eof", "%%%%*", None, None, None)),
    "err_norm_junk": (["spkA_u1=d/fb.fea"], 1, 0, 0, "ANON", False, None, ("norm/bad/junk", "%%%%*", None, None, None)),
    "err_norm_word": (["spkA_u1=d/fb.fea"], 1, 0, 0, "ANON", False, None, ("norm/bad/word", "%%%%*", None, None, None)),
    "err_norm_cvn_missing": (["spkA_u1=d/fb.fea"], 1, 0, 0, "ANON", False, None,
                             (None, None, "norm/nosuch", "%%%%*", None)),
}


def run_harness(td, scp, swap, sext, eext, tk, mlf, ldir, out, norm=None):
    os.makedirs(out, exist_ok=True)
    cmd = [HARNESS, "features", scp, str(swap), str(sext), str(eext), tk, mlf or "-", "states.txt", ldir or "-", "lab",
           out] + ([v or "-" for v in norm] if norm else [])
    subprocess.run(cmd, cwd=td, check=True, capture_output=True)
    res = []
    for line in open(os.path.join(out, "index.txt")):
        k, rest = line.rstrip("\n").split(" ", 1)
        if rest.startswith("ERROR "):
            msg = rest[6:].split(" THE STACKTRACE")[0]
            if msg.startswith("ERROR ("):
                msg = msg[6:]
            if msg.startswith("(") and ") " in msg:  # KaldiLib's "(function:file:line) " prefix
                msg = msg.split(") ", 1)[1]
            res.append({"error": msg.strip()})
            continue
        rows, cols, per, kind, nl, logical = rest.split(" ", 5)
        rows, cols, nl = int(rows), int(cols), int(nl)
        x = np.fromfile(os.path.join(out, f"f{k}.f32"), np.float32).reshape(rows, cols)
        lab = np.fromfile(os.path.join(out, f"l{k}.i32"), np.int32) if nl else np.zeros(0, np.int32)
        res.append({"rows": rows, "cols": cols, "period": int(per), "kind": int(kind), "logical": logical, "x": x,
                    "lab": lab})
    return res


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build oracle/_ref first (make -C oracle ref)")
    rng = np.random.default_rng(7)
    files, mlf, states = synthetic(rng)
    arrays, meta = {}, {"configs": {}, "files": sorted(files)}
    for n, b in files.items():
        arrays[f"file:{n}"] = np.frombuffer(b, np.uint8)
    arrays["mlf"] = np.frombuffer(mlf.encode(), np.uint8)
    arrays["states"] = np.frombuffer(states.encode(), np.uint8)
    arrays["mlf:lookup.mlf"] = np.frombuffer(lookup_mlf().encode(), np.uint8)
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, "d"))
        for n, b in files.items():
            open(os.path.join(td, "d", n), "wb").write(b)
        open(os.path.join(td, "fb.fea"), "wb").write(files["fb.fea"])
        open(os.path.join(td, "test.mlf"), "w").write(mlf)
        open(os.path.join(td, "lookup.mlf"), "w").write(lookup_mlf())
        open(os.path.join(td, "states.txt"), "w").write(states)
        nf = norm_files(np.random.default_rng(11))
        for rel, text in nf.items():
            os.makedirs(os.path.join(td, os.path.dirname(rel)), exist_ok=True)
            open(os.path.join(td, rel), "w").write(text)
            arrays[f"norm:{rel}"] = np.frombuffer(text.encode(), np.uint8)
        for name, cfg in CONFIGS.items():
            lines, swap, sext, eext, tk, use_mlf, ldir = cfg[:7]
            norm = cfg[7] if len(cfg) > 7 else None
            scp = os.path.join(td, f"{name}.scp")
            open(scp, "w").write("\n".join(lines) + "\n")
            mlf_name = use_mlf if isinstance(use_mlf, str) else ("test.mlf" if use_mlf else None)
            res = run_harness(td, scp, swap, sext, eext, tk, mlf_name, ldir, os.path.join(td, "out_" + name), norm)
            cm = {"scp": lines, "swap": swap, "start_ext": sext, "end_ext": eext, "target_kind": tk,
                  "mlf": use_mlf, "label_dir": ldir, "norm": list(norm) if norm else None, "records": []}
            for k, r in enumerate(res):
                if "error" in r:
                    cm["records"].append({"error": r["error"]})
                    continue
                cm["records"].append({kk: r[kk] for kk in ("rows", "cols", "period", "kind", "logical")})
                arrays[f"{name}:x{k}"] = r["x"]
                arrays[f"{name}:lab{k}"] = r["lab"]
            meta["configs"][name] = cm
        # examples/01, first 20 utterances, the run_test recipe's 25 / 25 frame extension
        ex_lines = [l.strip() for l in open(os.path.join(EX, "test.scp")) if l.strip()][:20]
        scp = os.path.join(td, "ex01.scp")
        open(scp, "w").write("\n".join(os.path.join(EX, l) for l in ex_lines) + "\n")
        for f in ("test_3s.mlf", "mono_state_phn_set_135_phn"):
            os.symlink(os.path.join(EX, f), os.path.join(td, f))
        out = os.path.join(td, "out_ex01")
        os.makedirs(out)
        subprocess.run([HARNESS, "features", scp, "1", "25", "25", "ANON", "test_3s.mlf", "mono_state_phn_set_135_phn",
                        "-", "lab", out], cwd=td, check=True, capture_output=True)
        recs = []
        for line in open(os.path.join(out, "index.txt")):
            k, rows, cols, per, kind, nl, logical = line.split()
            x = np.fromfile(os.path.join(out, f"f{k}.f32"), np.float32)
            lab = np.fromfile(os.path.join(out, f"l{k}.i32"), np.int32)
            recs.append({"utt": ex_lines[int(k)], "rows": int(rows), "cols": int(cols), "period": int(per),
                         "kind": int(kind), "sha256": hashlib.sha256(x.tobytes()).hexdigest()})
            arrays[f"ex01:lab{k}"] = lab
        meta["ex01"] = {"start_ext": 25, "end_ext": 25, "records": recs}
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "reader.npz"), **arrays)
    print(json.dumps({k: [r.get("error", r.get("rows")) for r in v["records"]] for k, v in meta["configs"].items()},
                     indent=1))


if __name__ == "__main__":
    main()
