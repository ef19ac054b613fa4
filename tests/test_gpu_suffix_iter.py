"""find_iter under MatchType::DfaSuffix over few long haystacks
(match_types.hip launch_suffix_iter): the reference's iteration is a chain
of exec_dfa_reverse_suffix searches (exec.rs:725-794), each from the
previous match end; with a suffix that cannot overlap itself every search
starts at an occurrence end, so each occurrence's slice is scanned once and
the searches the iteration makes are found by pointer doubling.  Against the
oracle's find_iter (the reference's search chain restated), including the
walk's quirk (`xa*ingb*ing|a+ing`) and the None fallbacks ("singing":
a reverse scan reaching its slice start).  rure_amd_last_fwd_path() == -11
asserts the path ran."""
import os

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex
from golden_data import corpus

pytestmark = pytest.mark.gpu

WORDS = [b"singing", b"ringing", b"bring", b"king ", b"ann@gmail.com", b"x@gmail.com", b"thing", b"ing",
         b"xaaingbing", b"xaing", b"aing ", b" ", b"\n", b"sing\xc3\xa9ing", b"inging"]
PATS = [r"[a-z]+ing", r"\w+@gmail\.com", r"xa*ingb*ing|a+ing", r"(?-u)[a-z]*\bing"]


def _text(n, seed):
    rng = np.random.default_rng(seed)
    base = corpus("sherlock")
    out = bytearray()
    while len(out) < n:
        if rng.integers(0, 2) == 0:
            out += WORDS[int(rng.integers(len(WORDS)))]
        else:
            a = int(rng.integers(0, len(base) - 120))
            out += base[a:a + int(rng.integers(1, 120))]
    return bytes(out[:n])


def _check(cuda, pat, count, L, seed, start=0, capacity=None):
    import torch
    text = b"".join(_text(L, seed + i) for i in range(count))
    d = torch.from_numpy(np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    re = R.Regex(pat)
    assert re.match_info()["match_type"] == "DfaSuffix", pat
    o = OracleRegex(re)
    counts, m = re.find_iter_batch(d, stride=L, length=L, count=count, start=start, capacity=capacity)
    assert N.rure_amd_last_fwd_path() == -11, pat
    counts = counts.cpu().numpy().tolist()
    got = [tuple(x) for x in m.cpu().numpy().tolist()]
    exp_all = []
    for h in range(count):
        exp = o.find_iter(text[h * L:(h + 1) * L], start)
        assert counts[h] == len(exp), (pat, h, counts[h], len(exp))
        exp_all += exp
    if capacity is None:
        assert got == exp_all, pat
    else:
        assert got == exp_all[:capacity], pat
    return len(exp_all)


@pytest.mark.parametrize("pat", PATS)
def test_suffix_iter_long(cuda, pat):
    assert _check(cuda, pat, 1, 600_000, 3) > 0


@pytest.mark.parametrize("pat", PATS)
@pytest.mark.parametrize("start", [0, 7])
def test_suffix_iter_small_units(cuda, pat, start):
    """units of 128 bytes: occurrences and slices cross many unit edges"""
    with R.debug(suffix_iter=2):
        for seed in range(3):
            _check(cuda, pat, 3, 9_000 + 177 * seed, 50 + seed, start)


def test_suffix_iter_quit_falls_back(cuda):
    r"""Unicode \b (a DFA that can quit): ASCII text stays on the parallel
    path; a non-ASCII byte next to a slice makes it give up to the wave path
    (its Pike VM answers), with the same results as the oracle"""
    import torch
    pat = r"\bx[a-z]*ing"
    re = R.Regex(pat)
    assert re.match_info()["match_type"] == "DfaSuffix"
    o = OracleRegex(re)
    L = 300_000
    text = bytearray(_text(L, 77).replace(b"\xc3\xa9", b"ee"))
    text = bytes(b if b < 0x80 else 0x20 for b in text)
    for t in (text, text[:1000] + "é".encode() + b"xaing " + text[1008:]):
        t = t[:L]
        d = torch.from_numpy(np.frombuffer(t + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
        counts, m = re.find_iter_batch(d, stride=L, length=L, count=1)
        got = [tuple(x) for x in m.cpu().numpy().tolist()]
        assert got == o.find_iter(t), pat
        if t == text:
            assert N.rure_amd_last_fwd_path() == -11, pat


def test_suffix_iter_capacity_and_empty(cuda):
    import torch
    with R.debug(suffix_iter=2):
        n = _check(cuda, PATS[0], 2, 20_000, 9)
        _check(cuda, PATS[0], 2, 20_000, 9, capacity=n // 3)
        # no occurrence at all
        re = R.Regex(PATS[0])
        text = b"x" * 5000
        d = torch.from_numpy(np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
        counts, m = re.find_iter_batch(d, stride=5000, length=5000, count=1)
        assert counts.cpu().numpy().tolist() == [0] and m.shape[0] == 0
