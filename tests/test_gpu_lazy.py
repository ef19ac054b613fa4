"""The on-demand forward DFA (host LazyDfa, big_dfa.hip lazy_dfa_kernel):
rows are built when a scan first needs them, as the reference's lazy DFA
builds a state when a search first steps into it (dfa.rs:910-1048); lanes
that meet a missing row park, the host builds the rows and the next round
resumes them.  `(?:a|b)*a(?:a|b){20}` has ~2^21 states, past the eager
budgets (kBigDfaRawStates), so it used to run on the Pike VM; debug knobs
lazy=1, lazy_rows=1 (one row built ahead per round) force ordinary
regexes through many parking rounds.  find / is_match / shortest_match
against the oracle; rure_amd_last_fwd_path() == -10 asserts the lazy kernel
answered."""
import os

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex
from golden_data import corpus

pytestmark = pytest.mark.gpu

HUGE = r"(?:a|b)*a(?:a|b){20}"


def _mixed(n, L, seed):
    """sherlock lines with runs of a/b of random lengths (some past 21)"""
    rng = np.random.default_rng(seed)
    base = corpus("sherlock")
    out = bytearray()
    while len(out) < n * L:
        if rng.integers(0, 3) == 0:
            out += bytes(rng.choice(np.frombuffer(b"ab", dtype=np.uint8), size=int(rng.integers(1, 40))))
        else:
            a = int(rng.integers(0, len(base) - 100))
            out += base[a:a + int(rng.integers(1, 100))]
    return bytes(out[:n * L])


def _check(cuda, pat, raw, n, L, start=0):
    import torch
    d = torch.from_numpy(np.frombuffer(raw + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    re = R.Regex(pat)
    o = OracleRegex(re)
    got_f = re.find_batch(d, stride=L, length=L, count=n, start=start).cpu().numpy()
    if re.match_info()["match_type"] == "Dfa":  # (literal / suffix match types run their own engines)
        assert N.rure_amd_last_fwd_path() == -10, pat
    got_m = re.is_match_batch(d, stride=L, length=L, count=n, start=start).cpu().numpy()
    got_s = re.shortest_match_batch(d, stride=L, length=L, count=n, start=start).cpu().numpy()
    hits = 0
    for i in range(n):
        h = raw[i * L:(i + 1) * L]
        e = o.find(h, start)
        g = None if got_f[i, 0] < 0 else (int(got_f[i, 0]), int(got_f[i, 1]))
        assert g == e, (pat, i, g, e)
        assert bool(got_m[i]) == o.is_match(h, start), (pat, i)
        es = o.shortest_match(h, start)
        assert (None if got_s[i] < 0 else int(got_s[i])) == es, (pat, i)
        hits += e is not None
    return hits


@pytest.mark.parametrize("start", [0, 3])
def test_lazy_huge(cuda, start):
    """past the eager budgets: the lazy kernel, not the Pike VM"""
    n, L = 400, 200
    with R.debug(big=2):
        hits = _check(cuda, HUGE, _mixed(n, L, 5 + start), n, L, start)
    assert 0 < hits < n


@pytest.mark.parametrize("pat", [r"\d{4}-\d{2}-\d{2}", r"[a-z]+ing", r"Sherlock|Holmes", r"(?i)holmes\w*",
                                 r"(?-u)\bthe\b", r"x*", r"(?s).{3}$|^Th", HUGE])
def test_lazy_forced_rounds(cuda, pat):
    """one row built ahead per round: every lane parks many times"""
    n, L = 300, 150
    raw = _mixed(n, L, len(pat))
    with R.debug(lazy=1, lazy_rows=1):
        _check(cuda, pat, raw, n, L, 0)


def test_lazy_offsets(cuda):
    import torch
    re = R.Regex(HUGE)
    o = OracleRegex(re)
    rng = np.random.default_rng(11)
    text = _mixed(1, 60000, 3)
    cuts = np.sort(rng.choice(len(text), size=500, replace=False))
    offs = np.concatenate([[0], cuts, [len(text)]]).astype(np.int64)
    d = torch.from_numpy(np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    with R.debug(big=2):
        got = re.find_batch(d, offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy()
        assert N.rure_amd_last_fwd_path() == -10
    for i in range(len(offs) - 1):
        h = text[offs[i]:offs[i + 1]]
        e = o.find(h)
        g = None if got[i, 0] < 0 else (int(got[i, 0]), int(got[i, 1]))
        assert g == e, i
