"""GPU parity: HIP kernels (through the C ABI) vs the CPU oracle, bit-exact."""
import numpy as np
import pytest

import regex_amd as R
from oracle_py import OracleRegex
from regex_amd.workloads import date_haystacks_host

pytestmark = pytest.mark.gpu

PATTERNS = [
    r"\d{4}-\d{2}-\d{2}",
    r"\w+@\w+\.\w+",
    r"a+",
    r"(?i)sherlock|holmes",
    r"[a-z]{3}\d",
    r"x*",
    r"^\d",
    r"\d$",
    r"(?m)^\d+$",
    r"(?-u)\bab\b",
    r"",
]


def _to_dev(buf, cuda):
    import torch
    return torch.from_numpy(buf).to(cuda)


@pytest.mark.parametrize("pat", PATTERNS)
def test_find_batch_strided(cuda, pat):
    n, L = 2048, 257
    buf, _ = date_haystacks_host(n, L, seed=11, frac=0.05)
    re = R.Regex(pat)
    o = OracleRegex(re)
    dev = _to_dev(buf, cuda)
    got = re.find_batch(dev, stride=L, length=L, count=n).cpu().numpy().astype(np.uint64)
    ism = re.is_match_batch(dev, stride=L, length=L, count=n).cpu().numpy()
    sho = re.shortest_match_batch(dev, stride=L, length=L, count=n).cpu().numpy().astype(np.uint64)
    for i in range(n):
        t = bytes(buf[i * L:(i + 1) * L])
        exp = o.find(t)
        g = None if int(got[i, 0]) == R.NONE else (int(got[i, 0]), int(got[i, 1]))
        assert g == exp, (pat, i, g, exp)
        assert bool(ism[i]) == (exp is not None)
        es = o.shortest_match(t)
        gs = None if int(sho[i]) == R.NONE else int(sho[i])
        assert gs == es, (pat, i, gs, es)


@pytest.mark.parametrize("pat", [r"\d{4}-\d{2}-\d{2}", r"[a-z]{3}\d", r"\w+@\w+\.\w+", r"(?m)^\d+$", "x*"])
@pytest.mark.parametrize("n,L,stride", [(1000, 4096, 4096), (333, 1000, 1008), (64, 128, 128), (130, 300, 304)])
def test_find_batch_tiles(cuda, pat, n, L, stride):
    """Fixed-stride batches that take the coalesced-tile kernel (stride % 16 == 0)."""
    import torch
    buf2, _ = date_haystacks_host(n, stride, seed=7, frac=0.2)
    # plant dates straddling 128-byte tile boundaries
    for i in range(0, n, 5):
        o = i * stride + min(L - 10, 123 + (i % 7))
        buf2[o:o + 10] = np.frombuffer(b"1999-12-31", dtype=np.uint8)
    re = R.Regex(pat)
    o = OracleRegex(re)
    dev = torch.from_numpy(buf2).to(cuda)
    got = re.find_batch(dev, stride=stride, length=L, count=n).cpu().numpy()
    ism = re.is_match_batch(dev, stride=stride, length=L, count=n).cpu().numpy()
    sho = re.shortest_match_batch(dev, stride=stride, length=L, count=n).cpu().numpy()
    for i in range(n):
        t = bytes(buf2[i * stride:i * stride + L])
        exp = o.find(t)
        g = None if int(got[i, 0]) == -1 else (int(got[i, 0]), int(got[i, 1]))
        assert g == exp, (pat, i, g, exp)
        assert bool(ism[i]) == (exp is not None)
        es = o.shortest_match(t)
        assert (None if int(sho[i]) == -1 else int(sho[i])) == es


def test_find_batch_ragged(cuda):
    import torch
    rng = np.random.default_rng(5)
    n = 3000
    lens = rng.integers(0, 300, size=n)
    buf, _ = date_haystacks_host(1, int(lens.sum()) + 64, seed=3, frac=0.0)
    # plant some dates
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    for i in range(0, n, 7):
        if lens[i] >= 10:
            o = offs[i] + rng.integers(0, lens[i] - 9)
            buf[o:o + 10] = np.frombuffer(b"2024-02-29", dtype=np.uint8)
    re = R.Regex(r"\d{4}-\d{2}-\d{2}")
    o = OracleRegex(re)
    got = re.find_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy()
    for i in range(n):
        t = bytes(buf[offs[i]:offs[i + 1]])
        exp = o.find(t)
        g = None if int(got[i, 0]) == -1 else (int(got[i, 0]), int(got[i, 1]))
        assert g == exp, (i, g, exp)


def test_single_call_api(cuda):
    re = R.Regex(r"\d{4}-\d{2}-\d{2}")
    assert re.find(b"on 2017-12-30, then") == (3, 13)
    assert re.is_match(b"2017-12-30")
    assert not re.is_match(b"2017-12-3")
    assert re.find_iter(b"2017-12-30 2018-01-01") == [(0, 10), (11, 21)]
    assert R.Regex(r"").find_iter(b"ab") == [(0, 0), (1, 1), (2, 2)]


def test_set_batch(cuda):
    import torch
    pats = ["foo", "oo", r"\d+", "^x", "z$"]
    s = R.RegexSet(pats)
    o = OracleRegex(s)
    texts = [b"foo", b"x12", b"zzz", b"", b"xfooz", b"oo", b"abc"]
    L = 8
    buf = np.zeros(len(texts) * L, dtype=np.uint8)
    offs = np.zeros(len(texts) + 1, dtype=np.int64)
    pos = 0
    for i, t in enumerate(texts):
        buf[pos:pos + len(t)] = np.frombuffer(t, dtype=np.uint8) if t else []
        pos += len(t)
        offs[i + 1] = pos
    got = s.matches_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy()
    for i, t in enumerate(texts):
        exp = o.matches(t)
        g = [j for j in range(len(pats)) if (int(got[i]) >> j) & 1]
        assert g == exp, (t, g, exp)
        assert s.matches(t) == exp
