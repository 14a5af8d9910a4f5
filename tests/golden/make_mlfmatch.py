"""Golden vectors for the label masks and the MLF record index (csrc/host/labelindex.{h,cpp}): the reference's own
KaldiLib ProcessMask (src/KaldiLib/StkMatch.cc:453-490, over matche / matche_after_star) and LabelContainer
Insert / Find (src/KaldiLib/MlfStream.cc:43-265), built here by oracle/Makefile.ref and driven through
oracle/_ref/ref_harness `mlfmatch`.

  masks   : random masks over the mask alphabet ('*', '?', '%', sets with '!' / '^', ranges, '\\' escapes,
            malformed sets included) against random labels, plus the shapes TNetCu configurations use
            ("%%%%*", "*/spk%%%_*.fea", ...); expected: match or not, and the '%' captures
  lookups : random MLF record lists (exact names, "*/"-led names of several directory depths, "*name",
            names without a leading '/', wildcard patterns) inserted in order, then labels looked up;
            expected: the record number or -1

Writes tests/golden/mlfmatch.npz (one JSON document).  Run in the build container (needs /root/reference
and `make -C oracle -f Makefile.ref _ref/ref_harness`); the test never needs the reference.
"""
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")

MASK_ALPHA = list("ab/.") * 3 + list("*?%[]!^-\\c")
TEXT_ALPHA = list("ab/.") * 3 + list("c-]\\%*")


def rand_str(rng, alpha, lo, hi):
    return "".join(rng.choice(alpha) for _ in range(int(rng.integers(lo, hi + 1))))


def rand_set(rng):
    body = ""
    for _ in range(int(rng.integers(0, 4))):
        c = str(rng.choice(list("ab.c/]-\\")))
        if rng.random() < 0.4:
            body += c + "-" + str(rng.choice(list("abc.\\]")))
        else:
            body += c
    neg = str(rng.choice(["", "", "!", "^"]))
    close = "]" if rng.random() < 0.85 else ""
    return "[" + neg + body + close


def rand_mask(rng):
    parts = []
    for _ in range(int(rng.integers(0, 6))):
        r = rng.random()
        if r < 0.25:
            parts.append(rand_set(rng))
        else:
            parts.append(rand_str(rng, MASK_ALPHA, 1, 3))
    return "".join(parts)


def mask_cases(rng):
    cases = []
    fixed_masks = ["%%%%*", "%%%%?*", "*/spk%%%_*.fea", "*", "", "*/*", "%*", "*%", "a*", "*.lab", "**",
                   "*/a/*.lab", "[a-c]*", "*[!a]", "*[^/]*", "*\\", "[]a", "[a-]", "[\\]]*", "*?%*%?"]
    fixed_texts = ["spkA_u1", "/x/spkB_1.fea", "a.lab", "/a/b.lab", "ab", "", "/", "a", "b/a.lab", "\\a\\b.lab"]
    for m in fixed_masks:
        for t in fixed_texts:
            cases.append((m, t))
    for _ in range(12000):
        m = rand_mask(rng)
        t = rand_str(rng, TEXT_ALPHA, 0, 9)
        if rng.random() < 0.3 and m:  # a text built to come close to the mask
            t = "".join(c if c not in "*?%[]!^\\" else str(rng.choice(list("ab/."))) for c in m)
        cases.append((m, t))
    return cases


def rand_path(rng, seps="/"):
    comps = [rand_str(rng, list("ab"), 1, 2) for _ in range(int(rng.integers(0, 4)))]
    sep = str(rng.choice(list(seps)))
    lead = sep if rng.random() < 0.7 else ""
    return lead + sep.join(comps + [rand_str(rng, list("ab"), 1, 2) + ".lab"])


def lookup_cases(rng):
    boxes = []
    for _ in range(700):
        pats = []
        for _ in range(int(rng.integers(1, 9))):
            p = rand_path(rng, "/\\" if rng.random() < 0.15 else "/")
            r = rng.random()
            if r < 0.3:
                comps = p.lstrip("/\\").split("/")
                p = "*/" + "/".join(comps[int(rng.integers(0, len(comps))):])
            elif r < 0.4:
                p = "*" + p.lstrip("/").split("/")[-1]
            elif r < 0.55:
                p = p[: int(rng.integers(1, len(p) + 1))] + str(rng.choice(["*", "?", "%", "*.lab"]))
                if rng.random() < 0.5:
                    p = "*/" + p.lstrip("/")
            pats.append(p)
        labels = [rand_path(rng, "/\\" if rng.random() < 0.15 else "/") for _ in range(12)]
        labels += [p.replace("*", "x").replace("?", "a").replace("%", "b") for p in pats]
        labels += ["/" + p.lstrip("*/") for p in pats if p.startswith("*")]
        boxes.append((pats, labels))
    return boxes


def main():
    rng = np.random.default_rng(20261018)
    masks = mask_cases(rng)
    boxes = lookup_cases(rng)
    lines = []
    for m, t in masks:
        lines.append(f"M\t{m}\t{t}")
    for pats, labels in boxes:
        lines.append("R")
        for k, p in enumerate(pats):
            lines.append(f"I\t{p}\t{k}")
        for x in labels:
            lines.append(f"F\t{x}")
    out = subprocess.run([HARNESS, "mlfmatch"], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         check=True).stdout.split("\n")
    pos = 0
    mask_res = []
    for m, t in masks:
        ans = out[pos]
        pos += 1
        mask_res.append([m, t, None if ans == "0" else ans.split("\t", 1)[1]])
    box_res = []
    for pats, labels in boxes:
        recs = [int(out[pos + i]) for i in range(len(labels))]
        pos += len(labels)
        box_res.append([pats, labels, recs])
    doc = {"masks": mask_res, "lookups": box_res}
    n_match = sum(r[2] is not None for r in mask_res)
    n_found = sum(sum(x >= 0 for x in b[2]) for b in box_res)
    print(f"{len(mask_res)} mask cases ({n_match} matches), {len(box_res)} indexes, "
          f"{sum(len(b[1]) for b in box_res)} lookups ({n_found} found)")
    np.savez_compressed(os.path.join(HERE, "mlfmatch.npz"), doc=np.frombuffer(json.dumps(doc).encode(), np.uint8))


if __name__ == "__main__":
    main()
