"""Automata past the u16 tables (more than 65535 states): the host builds
them in u32 column form (dfa_build.cpp, kBigDfaRawStates) and batched find /
is_match / shortest_match run them on big_dfa.hip's kernel — the reference's
find_dfa_forward (exec.rs:632-662) and shortest_dfa (exec.rs:692-694) over
the lazy DFA it would build on demand (dfa.rs:576-866).  Checked against the
oracle's lazy DFA (oracle/lazy_dfa.c) on the same inputs."""
import os

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

BIG = [r"[a-q][^u-z]{13}x", r"(?:a|b)*a(?:a|b){14}", r"(?i)[a-q][^u-z]{13}x"]


def _hay(n, L, seed, alphabet):
    rng = np.random.default_rng(seed)
    return rng.choice(np.frombuffer(alphabet, dtype=np.uint8), size=n * L).astype(np.uint8)


@pytest.fixture
def force_big():
    with R.debug(big=2):
        yield


@pytest.mark.parametrize("pat", BIG)
@pytest.mark.parametrize("start", [0, 5])
def test_big_batch_parity(cuda, force_big, pat, start):
    import torch
    n, L = 3000, 160
    alpha = b"abqxABQXuvz\n" if "a|b" not in pat else b"abc"
    buf = _hay(n, L, 0xB16 + start + len(pat), alpha)
    d = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(cuda)
    re = R.Regex(pat)
    o = OracleRegex(re)
    got_f = re.find_batch(d, stride=L, length=L, count=n, start=start).cpu().numpy()
    assert N.rure_amd_last_fwd_path() == -6
    got_m = re.is_match_batch(d, stride=L, length=L, count=n, start=start).cpu().numpy()
    got_s = re.shortest_match_batch(d, stride=L, length=L, count=n, start=start).cpu().numpy()
    raw = buf.tobytes()
    hits = 0
    for i in range(n):
        h = raw[i * L:(i + 1) * L]
        e = o.find(h, start)
        g = None if got_f[i, 0] < 0 else (int(got_f[i, 0]), int(got_f[i, 1]))
        assert g == e, (pat, i)
        assert bool(got_m[i]) == o.is_match(h, start), (pat, i)
        es = o.shortest_match(h, start)
        assert (None if got_s[i] < 0 else int(got_s[i])) == es, (pat, i)
        hits += e is not None
    assert 0 < hits < n


def test_big_offsets_and_empty(cuda, force_big):
    import torch
    pat = BIG[0]
    re = R.Regex(pat)
    o = OracleRegex(re)
    rng = np.random.default_rng(9)
    hs = [bytes(rng.choice(np.frombuffer(b"abqxuz", dtype=np.uint8), size=int(k)))
          for k in rng.integers(0, 90, size=700)]
    hs[3] = b""
    hs[7] = b"a" + b"b" * 13 + b"x"
    offs = np.cumsum([0] + [len(h) for h in hs]).astype(np.int64)
    d = torch.from_numpy(np.frombuffer(b"".join(hs) + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    got = re.find_batch(d, offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy()
    for i, h in enumerate(hs):
        e = o.find(h)
        g = None if got[i, 0] < 0 else (int(got[i, 0]), int(got[i, 1]))
        assert g == e, i
    assert got[7, 0] == 0 and got[7, 1] == 15


def test_big_default_threshold(cuda):
    """Without forcing: a batch that fills the device takes the big-DFA
    kernel; a small one (the Pike VM) gives the same answers."""
    import torch
    pat = BIG[0]
    re = R.Regex(pat)
    n, L = 20000, 64
    buf = _hay(n, L, 77, b"abqxuz")
    d = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(cuda)
    big = re.find_batch(d, stride=L, length=L, count=n).cpu().numpy()
    assert N.rure_amd_last_fwd_path() == -6
    small = re.find_batch(d, stride=L, length=L, count=200).cpu().numpy()
    assert (small == big[:200]).all()
