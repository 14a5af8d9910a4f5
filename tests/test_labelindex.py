"""Label masks and the MLF record index (csrc/host/labelindex.{h,cpp}; C ABI tnet_mask_match / tnet_mlf_lookup)
against the reference's own KaldiLib ProcessMask (src/KaldiLib/StkMatch.cc:453-490) and LabelContainer
Insert / Find (src/KaldiLib/MlfStream.cc:43-265), run here through oracle/_ref/ref_harness `mlfmatch`
(tests/golden/make_mlfmatch.py -> tests/golden/mlfmatch.npz): 12,200 masks x labels, malformed sets included,
and 700 random record lists with 13,291 lookups.

Tolerance: none -- match / no match, the '%' captures and the resolved record are exact.

Pure host code: runs on CPU (no device calls)."""
import json
import os

import numpy as np
import pytest

from tnet_amd import mask_match, mlf_lookup

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mlfmatch.npz")
DOC = json.loads(bytes(np.load(GOLD)["doc"]).decode())


def test_masks_match_reference_process_mask():
    bad = []
    for mask, label, want in DOC["masks"]:
        got = mask_match(mask, label)
        if got != want:
            bad.append((mask, label, want, got))
    assert not bad, f"{len(bad)} of {len(DOC['masks'])} differ, first: {bad[:5]}"


def test_lookups_match_reference_label_container():
    bad = []
    for pats, labels, want in DOC["lookups"]:
        got = mlf_lookup(pats, labels)
        for lab, w, g in zip(labels, want, got):
            if w != g:
                bad.append((pats, lab, w, g))
    assert not bad, f"{len(bad)} lookups differ, first: {bad[:5]}"


@pytest.mark.parametrize("mask,label,want", [
    ("%%%%*", "spkA_u1", "spkA"),          # the CMEANMASK idiom: the speaker prefix
    ("*/a*.lab", "/x/ab.lab", ""),
    ("[ab-]x]", "ax]", ""),                # a set that closes at the first ']' after the member 'a' ...
    ("[ab-]x]", "bx]", None),               # ... and is malformed for 'b' (the range "b-]")
    ("a**", "a", None),                    # the text ends under "**": only a lone final '*' matches nothing
    ("a*", "a", ""),
])
def test_mask_corner_cases(mask, label, want):
    assert mask_match(mask, label) == want
