r"""Unicode classes against Python's `re`, not against the product's front end
(tests/golden/gen_unicode_fixtures.py: stdlib `re` in str mode over code
points whose \w / \d / \s / L / case-fold membership agrees with the
reference's Unicode 10 tables).  The oracle runs the product's compiled
programs, so these fixtures are what catches a class the parser or the
tables got wrong on both sides.  Paths: the run engine (-19) for the C+
regexes, the per-line and per-lane kernels for ragged batches, the C2 tile
kernel (path 1, above 131,072 fixed-stride haystacks) and the chunked long
scan for C5's regex."""
import gzip
import json
import os

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
RUNS = [r"\w+", r"\pL+", r"\S+", r"\d+", r".+", r"(?i)[a-zé]+"]


def fixtures():
    with gzip.open(os.path.join(HERE, "golden", "unicode_re_fixtures.json.gz"), "rt", encoding="utf-8") as f:
        return json.load(f)


FX = fixtures()


def pairs(flat):
    return [(flat[i], flat[i + 1]) for i in range(0, len(flat), 2)]


def ragged(cuda, texts):
    import torch
    bs = [t.encode() for t in texts]
    offs = np.zeros(len(bs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(b) for b in bs])
    buf = np.frombuffer(b"".join(bs) + bytes(16), dtype=np.uint8)
    return torch.from_numpy(buf.copy()).to(cuda), torch.from_numpy(offs).to(cuda)


@pytest.mark.parametrize("pat", FX["patterns"])
def test_unicode_ragged_find_iter(cuda, pat):
    """find_iter over 300 ragged haystacks (0-3000 characters, empty ones
    included): every span, as UTF-8 byte offsets."""
    re = R.Regex(pat)
    buf, offs = ragged(cuda, FX["ragged"])
    counts, m = re.find_iter_batch(buf, offsets=offs)
    got = [tuple(x) for x in m.cpu().numpy().tolist()]
    exp_lists = [pairs(x) for x in FX["spans"][pat]["ragged"]]
    assert counts.cpu().numpy().tolist() == [len(x) for x in exp_lists]
    assert got == [s for x in exp_lists for s in x]


@pytest.mark.parametrize("pat", FX["patterns"])
def test_unicode_ragged_find(cuda, pat):
    """find / is_match over the same ragged batch (the per-line kernel)."""
    re = R.Regex(pat)
    buf, offs = ragged(cuda, FX["ragged"])
    got = re.find_batch(buf, offsets=offs).cpu().numpy()
    ism = re.is_match_batch(buf, offsets=offs).cpu().numpy()
    for i, flat in enumerate(FX["spans"][pat]["ragged"]):
        exp = (flat[0], flat[1]) if flat else None
        g = None if got[i, 0] < 0 else (int(got[i, 0]), int(got[i, 1]))
        assert g == exp, (i, g, exp)
        assert bool(ism[i]) == bool(flat)


@pytest.mark.parametrize("pat", FX["patterns"])
def test_unicode_long_find_iter(cuda, pat):
    """The two long haystacks (64 and 96 KiB of mixed 1-4 byte encodings) one
    at a time: chunked find_iter, and the run engine for the C+ regexes."""
    import torch
    re = R.Regex(pat)
    for text, flat in zip(FX["long"], FX["spans"][pat]["long"]):
        b = text.encode()
        d = torch.from_numpy(np.frombuffer(b + bytes(16), dtype=np.uint8).copy()).to(cuda)
        counts, m = re.find_iter_batch(d, stride=len(b), length=len(b), count=1)
        if pat in RUNS:
            assert N.rure_amd_last_fwd_path() == -19, pat
        assert int(counts[0]) == len(flat) // 2
        assert [tuple(x) for x in m.cpu().numpy().tolist()] == pairs(flat)


@pytest.mark.parametrize("pat", [r"\d{4}-\d{2}-\d{2}", r"\w+@\w+\.\w+", r"\pL+", r"\w+"])
def test_unicode_stride_tile(cuda, pat):
    """The 1024 fixed 256-byte haystacks repeated to 143,360 (above the
    131,072 threshold of the C2 tile kernel): the first match of each."""
    import torch
    L, rep = FX["stride_len"], 140
    one = b"".join(t.encode() for t in FX["stride"])
    assert len(one) == L * len(FX["stride"])
    n = len(FX["stride"]) * rep
    d = torch.from_numpy(np.frombuffer(one * rep + bytes(16), dtype=np.uint8).copy()).to(cuda)
    re = R.Regex(pat)
    got = re.find_batch(d, stride=L, length=L, count=n).cpu().numpy()
    if pat in (r"\d{4}-\d{2}-\d{2}", r"\w+@\w+\.\w+"):
        assert N.rure_amd_last_fwd_path() in (1, 2, 4), pat
    exp = np.array([x[:2] if x else [-1, -1] for x in FX["spans"][pat]["stride"]] * rep, dtype=np.int64)
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert bad.size == 0, (int(bad[0]), got[bad[0]].tolist(), exp[bad[0]].tolist())


@pytest.mark.parametrize("where", [0, 1])
def test_unicode_long_scan_email(cuda, where):
    """C5's regex over one 4 MiB haystack (the chunked long scan): ragged
    fixture texts with their '@' removed (no match can form), then a newline
    and one long fixture text; the first match is that text's first span,
    shifted."""
    import torch
    filler = "".join(t.replace("@", " ") for t in FX["ragged"])
    reps = (4 << 20) // len(filler.encode()) + 1
    head = (filler * reps + "\n").encode()
    tail = FX["long"][where].encode()
    flat = FX["spans"][r"\w+@\w+\.\w+"]["long"][where]
    b = head + tail
    d = torch.from_numpy(np.frombuffer(b + bytes(16), dtype=np.uint8).copy()).to(cuda)
    re = R.Regex(r"\w+@\w+\.\w+")
    got = re.find_batch(d, stride=len(b), length=len(b), count=1).cpu().numpy()
    assert (int(got[0, 0]), int(got[0, 1])) == (len(head) + flat[0], len(head) + flat[1])
    assert bool(re.is_match_batch(d, stride=len(b), length=len(b), count=1).cpu().numpy()[0])
