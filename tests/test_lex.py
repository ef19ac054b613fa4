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
from lex_sim import lex16, lex16x4, lex_unit, lex_walk
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


@pytest.mark.parametrize("pat", LEX_PATTERNS + [r"B", r"Y"])
def test_lex4_blocks_equal_bytes(pat):
    """build_lex4: four bytes per step gives the byte lexer's flag words and
    states on ASCII blocks, full and partial (the IUB codes' one-byte
    regexes too)."""
    re = R.Regex(pat)
    lex, lex4 = re.lex_table(), re.lex4_table()
    assert lex is not None and lex4 is not None, pat
    tab4, r0 = lex4
    # the row of each byte-table entry, followed along the walk
    rng = random.Random(zlib.crc32(pat.encode()))
    for i in range(40):
        t = ascii_text(rng.randrange(1 << 30), 16 * 40)
        if i % 3 == 2:
            t = bytes(rng.randrange(128) for _ in range(16 * 40))
        s, r = lex[1], r0
        ent_of_row = {r0: s}
        for bp in range(0, len(t), 16):
            kend = 16 if bp + 16 < len(t) or i % 2 == 0 else 1 + rng.randrange(16)
            blk = t[bp:bp + 16]
            m1, s = lex16(lex, s, blk, kend)
            m4, r = lex16x4(lex4, r, blk, kend)
            assert m1 == m4, (pat, i, bp, kend)
            assert ent_of_row.setdefault(r, s) == s, (pat, i, bp)
            if kend < 16:
                break


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
