"""CPU check of the chunked find_iter algorithm (iter_scan.hip, mirrored by
tests/iter_sim.py) over the find_iter DFA with stripped states: with tiny
chunks (many boundaries, matches straddling cuts) the result must equal the
oracle's sequential find_iter (re_trait.rs:197-221) exactly."""
import random
import zlib

import pytest

import regex_amd as R
from iter_sim import find_iter_chunked
from oracle_py import OracleRegex

PATTERNS = [r"a+", r"ab|a", r"[a-c]+d?", r"x*", r"(?s).", r"\w+@\w+\.\w+", r"\d{4}-\d{2}-\d{2}",
            r"agggtaaa|tttaccct", r"[cgt]gggtaaa|tttaccc[acg]", r">[^\n]*\n|\n", r"a*?b", r"(a|ab)(c|bcd)(d*)",
            r"[ab]{2,5}", r"", r"b*"]


def text(seed, n):
    rng = random.Random(seed)
    alpha = b"aabbcd x@.\n>0123-gt"
    return bytes(rng.choice(alpha) for _ in range(n))


@pytest.mark.parametrize("pat", PATTERNS)
@pytest.mark.parametrize("chunk", [7, 16, 61])
@pytest.mark.parametrize("slots", [2, 1 << 30])
def test_chunked_iter_matches_oracle(pat, chunk, slots):
    re = R.Regex(pat)
    assert re.nfa_tables()[0]["looks"] == 0
    fwd = re.dfa_tables(2)
    rev = re.dfa_tables(1)
    o = OracleRegex(re)
    for i in range(6):
        t = text(zlib.crc32(pat.encode()) + i, 150 + 37 * i)
        exp = o.find_iter(t)
        got = find_iter_chunked(fwd, rev, t, chunk, slots=slots)
        assert got == exp, (pat, chunk, i)


def test_strip_states_exist():
    info = R.Regex(r"\w+@\w+\.\w+").dfa_info(2)
    base = R.Regex(r"\w+@\w+\.\w+").dfa_info(0)
    assert info["ok"] == 1 and info["states"] >= base["states"]


FB_PATTERNS = [r">[^\n]*\n|\n", r"a+", r"a[^b]*b", r"[ab]c*", r"\n", r">[^\n]*", r"(?-u)>[^\n]*\n|\n",
               r"a(b|cd)*e?", r"ab*|ac*", r"(?s)a.*b|c"]


def mixed_text(seed, n):
    rng = random.Random(seed)
    alpha = [b"a", b"b", b"c", b"d", b"e", b"\n", b">", b"x", "é".encode(), b"\xff", b"\x80"]
    w = [8, 6, 5, 3, 2, 4, 3, 6, 1, 1, 1]
    return b"".join(rng.choices(alpha, weights=w, k=n))


@pytest.mark.parametrize("pat", FB_PATTERNS)
def test_first_byte_rule(pat):
    """The first-byte start rule (iter_scan.hip / host first_byte_rule): where
    the host says it holds, every cut-bounded search from every start that
    ends in the dead state over ASCII bytes starts at the first F byte — the
    same match the reverse scan finds."""
    re = R.Regex(pat)
    fb = re.first_bytes()
    assert fb, pat
    fwd = re.dfa_tables(2)
    rev = re.dfa_tables(1)
    o = OracleRegex(re)
    from dfa_sim import find
    used = 0
    for i in range(5):
        t = mixed_text(zlib.crc32(pat.encode()) + i, 120) if i % 2 else text(i, 120)
        for st in range(len(t) + 1):
            for cut in (None, st + 1, st + 5, st + 40):
                a = find(fwd, rev, t, st, cut=cut)
                b = find(fwd, rev, t, st, cut=cut, fb=fb)
                assert a == b, (pat, i, st, cut, a, b)
                used += a is not None
        assert find_iter_chunked(fwd, rev, t, 13, fb=fb) == o.find_iter(t)
    assert used > 50


def test_first_byte_rule_rejects():
    for pat in [r"abc|ab", r"\w+", r"\d{4}-\d{2}-\d{2}", r"x*", r"agggtaaa|tttaccct", r"a\b"]:
        assert R.Regex(pat).first_bytes() is None, pat


LOOK_PATTERNS = [r"(?-u)\b[a-c]+\b", r"(?-u)\bx", r"(?m)^a+", r"(?m)a+$", r"(?-u)a\B", r"(?-u)\B[ab]+", r"(?m)^$",
                 r"(?-u)\b", r"(?m)^", r"(?-u)[a-d]*\bd", r"a+\z", r"(?-u)\b\w+@\w+", r"(?-u)\B\w+",
                 r"(?-u)[a-c]*\B[ab]", r"(?m)a*^b", r"(?-u)\B", r"(?-u)\B[a-d]*\b", r"(?m)(?-u)$|\b",
                 r"(?-u)\b|\B[ab]", r"(?-u)[a-d]\B|x", r"(?m)[ab]*$", r"(?m)^[^\n]*$", r"(?m)^>.*$",
                 r"(?-u)\bd\b|\Ba", r"(?m)(?-u)^\w*\b"]


@pytest.mark.parametrize("pat", LOOK_PATTERNS)
def test_chunked_iter_look_around(pat):
    """Look-around: a search's reverse scan over [p, e) reads the slice start
    p as the text's start (exec.rs:656-660 runs it over text[p..e]), so a
    speculation entered fresh at a unit's c0 is exact only when its first
    reverse scan died before c0 (else the unit is repaired from the true
    entry), a NoMatch from the reverse scan ends the whole iteration, and
    exits compare strictly ahead of such a unit."""
    re = R.Regex(pat)
    assert re.nfa_tables()[0]["looks"] != 0
    fwd = re.dfa_tables(2)
    rev = re.dfa_tables(1)
    o = OracleRegex(re)
    for i in range(12):
        t = (text if i % 2 else mixed_text)(zlib.crc32(pat.encode()) + i, 40 + 23 * i)
        exp = o.find_iter(t)
        for chunk in (1, 2, 3, 7, 16):
            assert find_iter_chunked(fwd, rev, t, chunk, looks=True) == exp, (pat, chunk, i)


UWB_PATTERNS = [r"\b", r"\B", r"\b\w", r"\w\b", r"\B[a-z]{2}", r"[a-z]+ed\b", r"\b\w+\b", r"\w+\B", r"\b\w+n\b",
                r"(?m)^\w+\b", r"\b|\B"]


def uwb_text(seed, n, every):
    """words with non-ASCII letters, marks, CJK, punctuation and invalid
    bytes about every `every` bytes"""
    rng = random.Random(seed)
    words = [b"the", b"then", b"seen", b"added", b"ran", b"a", b"in", b"x1", b"_n"]
    seps = [b" ", b", ", b".\n", b"-"]
    odd = ["é".encode(), "ñ".encode(), b"\xff", "中".encode(), "’".encode(), "ёn".encode(), "́".encode()]
    out = []
    k = 0
    while k < n:
        w = rng.choice(words)
        if rng.random() < 6.0 / every:
            w = w[: rng.randint(0, len(w))] + rng.choice(odd) + w[rng.randint(0, len(w)):]
        s = rng.choice(seps)
        out += [w, s]
        k += len(w) + len(s)
    return b"".join(out)[:n]


@pytest.mark.parametrize("pat", UWB_PATTERNS)
def test_chunked_iter_unicode_boundary_wave(pat):
    """The wave-served iteration of a Unicode word boundary (iter_scan.hip
    iter_wspec_kernel .. iter_wemit_kernel; the reference's DFA quits on any
    byte >= 0x80, dfa.rs:1487-1496, and that search runs on its NFA,
    exec.rs:485-487): quitting searches on the NFA bounded by the cut, a
    start after a byte >= 0x80 with no match before the cut decided by the
    unbounded DFA scan, units after such a byte unsure.  Against the
    oracle's sequential find_iter, tiny units, sparse and dense non-ASCII."""
    re = R.Regex(pat)
    fwd = re.dfa_tables(2)
    rev = re.dfa_tables(1)
    o = OracleRegex(re)
    for i, every in enumerate((8, 30, 300, 8, 30, 300)):
        t = uwb_text(zlib.crc32(pat.encode()) + i, 700 + 97 * i, every)
        exp = o.find_iter(t)
        for chunk in (3, 7, 16, 61):
            assert find_iter_chunked(fwd, rev, t, chunk, looks=True, nfa=o.find_nfa) == exp, (pat, chunk, i)
