"""MatchType::DfaSuffix over few long haystacks (match_types.hip
launch_suffix_long): exec_dfa_reverse_suffix (exec.rs:725-756) cut into
units by suffix occurrence, each slice's reverse scan run in parallel, the
first decisive slice per haystack, and the reference's fall-back to the
forward DFA (None: a reverse scan reached its slice start, e.g. "singing")
on the chunked forward scan.  find / is_match / shortest_match against the
oracle, which restates the reference's sequential walk; patterns whose
longest common suffix overlaps itself keep one lane per haystack.
rure_amd_last_fwd_path() == -9 asserts the unit path ran (for the forward
fallback the long scan's path code follows it)."""
import os

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex
from golden_data import corpus

pytestmark = pytest.mark.gpu

WORDS = [b"singing", b"ringing", b"bring", b"king", b"ann@gmail.com", b"x@gmail.com", b"thing", b"in", b"ing",
         b"ping ", b"  ", b"\n", b"sing\xc3\xa9ing", b"abab", b"xabababab "]


def _text(n, seed):
    rng = np.random.default_rng(seed)
    base = corpus("sherlock")
    out = bytearray()
    while len(out) < n:
        if rng.integers(0, 3) == 0:
            out += WORDS[int(rng.integers(len(WORDS)))]
        else:
            a = int(rng.integers(0, len(base) - 200))
            out += base[a:a + int(rng.integers(1, 200))]
    return bytes(out[:n])


def _check(cuda, pat, count, L, seed, expect_path=None):
    import torch
    text = b"".join(_text(L, seed + i) for i in range(count))
    buf = np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()
    d = torch.from_numpy(buf).to(cuda)
    re = R.Regex(pat)
    assert re.match_info()["match_type"] == "DfaSuffix"
    o = OracleRegex(re)
    got = re.find_batch(d, stride=L, length=L, count=count).cpu().numpy()
    path = N.rure_amd_last_fwd_path()
    ism = re.is_match_batch(d, stride=L, length=L, count=count).cpu().numpy()
    sho = re.shortest_match_batch(d, stride=L, length=L, count=count).cpu().numpy()
    for h in range(count):
        hay = text[h * L:(h + 1) * L]
        m = o.find(hay)
        exp = [-1, -1] if m is None else list(m)
        assert got[h].tolist() == exp, (pat, h, got[h].tolist(), exp)
        assert bool(ism[h]) == o.is_match(hay), (pat, h)
        s = o.shortest_match(hay)
        assert int(sho[h]) == (-1 if s is None else s), (pat, h, int(sho[h]), s)
    if expect_path is not None:
        assert path in expect_path, (pat, path)
    return got


@pytest.mark.parametrize("pat", [r"[a-z]+ing", r"\w+@gmail\.com"])
def test_suffix_long(cuda, pat):
    _check(cuda, pat, 3, 700_000, 11, expect_path=(-9, -4))  # -4: the forward fallback ran last
    _check(cuda, pat, 1, 4_000_000, 12)


@pytest.mark.parametrize("pat", [r"[a-z]+ing", r"\w+@gmail\.com"])
def test_suffix_long_small_units(cuda, pat):
    """units of 128 B (debug knob suffix_long=2): occurrences and slices
    cross many unit edges"""
    with R.debug(suffix_long=2):
        for seed in range(4):
            _check(cuda, pat, 3, 20_000 + 333 * seed, 40 + seed)


def test_suffix_long_no_occurrence(cuda):
    """no suffix occurrence at all, and one only at the very end"""
    import torch
    re = R.Regex(r"[a-z]+ing")
    o = OracleRegex(re)
    L = 300_000
    for tail in (b"", b"zing"):
        text = b"x" * (L - len(tail)) + tail
        d = torch.from_numpy(np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
        got = re.find_batch(d, stride=L, length=L, count=1).cpu().numpy()[0].tolist()
        m = o.find(text)
        assert got == ([-1, -1] if m is None else list(m)), tail


@pytest.mark.parametrize("pat", [r"[a-z]+ingi", r"\w+abab"])
def test_suffix_bordered_keeps_lanes(cuda, pat):
    """a self-overlapping lcs ("ingi", "abab"): the greedy occurrence walk is
    not every occurrence, so the lane search answers"""
    _check(cuda, pat, 2, 300_000, 21, expect_path=(-5,))


def test_suffix_walk_differs_from_forward(cuda):
    """The reference's suffix walk is not the forward DFA's leftmost-first
    search: `xa*ingb*ing|a+ing` over `xaaingbing` gives (1, 6) (the first
    "ing" decides: `a+ing` ends there), where a forward search gives (0, 10).
    Short haystacks (lane path) and a long one (units path) both follow the
    reference (the oracle restates its walk)."""
    import torch
    pat = r"xa*ingb*ing|a+ing"
    re = R.Regex(pat)
    o = OracleRegex(re)
    assert o.find(b"xaaingbing") == (1, 6)
    short = b"xaaingbing" + b" " * 22
    d = torch.from_numpy(np.frombuffer(short * 4 + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    got = re.find_batch(d, stride=len(short), length=len(short), count=4).cpu().numpy()
    assert got.tolist() == [[1, 6]] * 4
    L = 400_000
    text = b"z" * (L - 100) + b"xaaingbing" + b"q" * 90
    d = torch.from_numpy(np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    got = re.find_batch(d, stride=L, length=L, count=1).cpu().numpy()[0].tolist()
    assert got == list(o.find(text)) == [L - 99, L - 94]
    assert N.rure_amd_last_fwd_path() == -9
