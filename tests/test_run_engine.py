"""CPU check of the find_iter run engine's premise (host run_class,
run_iter.hip): for a regex detected as one byte class repeated (C+), the
reference's iteration (re_trait.rs:197-221, restated by the oracle) yields
exactly the maximal runs of C bytes — over all bytes for a class exact on
every byte, over ASCII text for a class whose bytes >= 0x80 quit.  Regexes
that are not C+ (lazy, bounded, anchored, look-around, sequences) must not
be detected."""
import random
import zlib

import numpy as np
import pytest

import regex_amd as R
from oracle_py import OracleRegex

RUNS = [r"\w+", r"[a-z]+", r"\S+", r"\pL+", r"\d+", r"(?-u)\w+", r"a+", r"[^\n]+", r".+", r"\s+",
        r"(?i)[a-f]+", r"(?s).+", r"[^a]+", r"[0-9A-Fa-f]+", r"(?:[a-c]|[x-z])+", r"[a-z][a-z]*", r"\w\w*"]
NOT_RUNS = [r"\w+?", r"(?:ab)+", r"a+b", r"\w{2,4}", r"\b\w+", r"(?m)^\w+", r"x*", r"[a-z]+ing", r"\w+\b",
            r"a|b+", r"[a-z]+[0-9]", r"\w{2,}", r"(?m)\w+$", r"\pL"]


def runs(cls, t):
    a = np.frombuffer(t, dtype=np.uint8)
    m = (cls[a] & 1).astype(bool)
    out, i, n = [], 0, len(t)
    while i < n:
        if m[i]:
            j = i
            while j < n and m[j]:
                j += 1
            out.append((i, j))
            i = j
        else:
            i += 1
    return out


def text(seed, n, nonascii):
    rng = random.Random(seed)
    alpha = [b"a", b"b", b"f", b"x", b"Z", b"0", b"9", b" ", b" ", b"\n", b"\t", b"_", b".", b"-", b"@"]
    if nonascii:
        alpha += ["é".encode(), "✓".encode(), b"\xff", "٣".encode()]
    return b"".join(rng.choices(alpha, k=n))[:n]


@pytest.mark.parametrize("pat", RUNS)
def test_run_class_detected_and_exact(pat):
    re = R.Regex(pat)
    cls = re.run_class()
    if cls is None:
        cls = re.run_class(ascii=True)
    assert cls is not None, pat
    o = OracleRegex(re)
    quits = bool(cls[0x80] & 2)
    for i in range(8):
        nonascii = not quits and i % 2 == 1
        t = text(zlib.crc32(pat.encode()) + i, 300 + 37 * i, nonascii)
        assert runs(cls, t) == o.find_iter(t), (pat, t)
        for st in (1, 5, 17):  # a search from start: runs of text[start:]
            exp = o.find_iter(t, st)
            got = [(a + st, b + st) for a, b in runs(cls, t[st:])]
            assert got == exp, (pat, st)


@pytest.mark.parametrize("pat", NOT_RUNS)
def test_not_runs(pat):
    re = R.Regex(pat)
    assert re.run_class() is None and re.run_class(ascii=True) is None, pat
