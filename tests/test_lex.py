"""CPU check of the find_iter lexer kernel's algorithm (tests/lex_sim.py
mirrors iter_spec_lex_tile_kernel) against the generic speculative
iteration of the same units (tests/iter_sim.py, iter_spec_burst_kernel):
identical matches, exits and clean flags for every unit, and the whole
chunked pipeline equal to the oracle's find_iter (re_trait.rs:197-221)."""
import random
import zlib

import numpy as np
import pytest

import regex_amd as R
from iter_sim import UnitIter, find_iter_chunked
from lex_sim import lex_unit, lex_walk
from oracle_py import OracleRegex

LEX_PATTERNS = [r">[^\n]*\n|\n", r"\n", r"a[^b]*b", r"(?-u)>[^\n]*\n|\n", r'"[^"]*"', r"<[^>]*>"]


def ascii_text(seed, n):
    rng = random.Random(seed)
    alpha = [b"a", b"b", b"c", b"g", b"t", b"\n", b">", b'"', b"<", b">", b" "]
    w = [6, 3, 3, 10, 10, 3, 1, 1, 1, 1, 3]
    return b"".join(rng.choices(alpha, weights=w, k=n))


def test_lex_tables_exist():
    for pat in LEX_PATTERNS:
        assert R.Regex(pat).lex_table() is not None, pat
    for pat in [r"a+", r">[^\n]*", r"\w+", r"\d{4}-\d{2}-\d{2}", r"x*", r"abc|ab"]:
        assert R.Regex(pat).lex_table() is None, pat


@pytest.mark.parametrize("pat", LEX_PATTERNS)
def test_lex_walk_whole_text(pat):
    """Without cuts the lexer alone is the iteration (ASCII text)."""
    re = R.Regex(pat)
    tab = re.lex_table()
    o = OracleRegex(re)
    for i in range(4):
        t = ascii_text(zlib.crc32(pat.encode()) + i, 700)
        ms, p, lm, frozen, _ = lex_walk(tab, t, 0, len(t))
        assert not frozen
        exp = o.find_iter(t)
        # matches ending before the end of the text (the kernel leaves the
        # search in progress at the end to the generic path)
        assert ms == [m for m in exp if m[1] < len(t)][:len(ms)]
        assert len(ms) >= len(exp) - 1


@pytest.mark.parametrize("pat", LEX_PATTERNS)
@pytest.mark.parametrize("chunk", [16, 48, 128])
def test_lex_units_equal_generic(pat, chunk):
    re = R.Regex(pat)
    tab = re.lex_table()
    fwd, rev = re.dfa_tables(2), re.dfa_tables(1)
    for i in range(3):
        t = ascii_text(zlib.crc32(pat.encode()) * 7 + i, 900)
        if i == 2:  # non-ASCII bytes: those units finish with the generic path
            t = t[:300] + "é".encode() + t[302:500] + b"\xff" + t[501:]
        nk = (len(t) + chunk - 1) // chunk
        for k in range(nk):
            c0, c1 = k * chunk, (1 << 62 if k + 1 == nk else (k + 1) * chunk)
            got = lex_unit(tab, fwd, rev, t, c0, c1)
            it = UnitIter(fwd, rev, t, (c0, None), c1)
            ms = []
            while True:
                m = it.next()
                if m is None:
                    break
                ms.append(m)
            assert got == (ms, it.exit, it.clean), (pat, chunk, i, k)
        assert find_iter_chunked(fwd, rev, t, chunk) == OracleRegex(re).find_iter(t)
