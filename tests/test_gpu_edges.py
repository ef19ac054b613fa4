"""Edge cases of the batched entry points on the GPU, against the oracle:
empty haystacks, search starts past the end, start > 0 on every path, sets
with a start offset, find_iter output truncation, empty batches and the
single-call API on empty input."""
import numpy as np
import pytest

import regex_amd as R
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

PATS = [r"\d{4}-\d{2}-\d{2}", r"a*", r"^b", r"b$", r"(?-u:\b)\w", r"x|yz", r""]


def ragged(texts):
    offs = np.zeros(len(texts) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(t) for t in texts])
    buf = np.frombuffer(b"".join(texts) + b"\0" * 16, dtype=np.uint8).copy()
    return buf, offs


TEXTS = [b"", b"a", b"b", b"ab", b"ba", b"2017-12-30", b"xx 2017-12-30 yz", b"\n", b"aaab", b"b b", b"yzx"]


@pytest.mark.parametrize("pat", PATS)
@pytest.mark.parametrize("start", [0, 1, 2, 5])
def test_ragged_all_apis_with_start(cuda, pat, start):
    import torch
    re = R.Regex(pat)
    o = OracleRegex(re)
    buf, offs = ragged(TEXTS)
    dev = torch.from_numpy(buf).to(cuda)
    doff = torch.from_numpy(offs).to(cuda)
    got = re.find_batch(dev, offsets=doff, start=start).cpu().numpy()
    ism = re.is_match_batch(dev, offsets=doff, start=start).cpu().numpy()
    sho = re.shortest_match_batch(dev, offsets=doff, start=start).cpu().numpy()
    for i, t in enumerate(TEXTS):
        exp = o.find(t, start) if start <= len(t) else None
        g = None if got[i, 0] < 0 else (int(got[i, 0]), int(got[i, 1]))
        assert g == exp, (pat, t, start)
        assert bool(ism[i]) == (o.is_match(t, start) if start <= len(t) else False), (pat, t, start)
        es = o.shortest_match(t, start) if start <= len(t) else None
        assert (None if sho[i] < 0 else int(sho[i])) == es, (pat, t, start)


@pytest.mark.parametrize("start", [0, 3, 200])
def test_strided_start_offsets(cuda, start):
    """Fixed-stride batches with start > 0 leave the tile path (start == 0 only)."""
    import torch
    from regex_amd.workloads import date_haystacks_host
    n, L = 300, 256
    buf, _ = date_haystacks_host(n, L, seed=21, frac=0.3)
    re = R.Regex(r"\d{4}-\d{2}-\d{2}")
    o = OracleRegex(re)
    got = re.find_batch(torch.from_numpy(buf).to(cuda), stride=L, length=L, count=n, start=start).cpu().numpy()
    for i in range(n):
        exp = o.find(bytes(buf[i * L:(i + 1) * L]), start)
        g = None if got[i, 0] < 0 else (int(got[i, 0]), int(got[i, 1]))
        assert g == exp


def test_set_with_start(cuda):
    import torch
    pats = ["^a", "a", r"\bb", "b$", "ab"]
    rs = R.RegexSet(pats)
    o = OracleRegex(rs)
    buf, offs = ragged(TEXTS)
    for start in (0, 1, 3):
        got = rs.matches_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda),
                               start=start).cpu().numpy()
        for i, t in enumerate(TEXTS):
            exp = o.matches(t, start) if start <= len(t) else []
            assert [j for j in range(len(pats)) if (int(got[i]) >> j) & 1] == exp, (t, start)


def test_find_iter_truncated_output(cuda):
    """capacity < total: counts and total stay exact, the first `capacity`
    records are written."""
    import torch
    text = b"a1 b22 c333 d4444 " * 50
    re = R.Regex(r"\d+")
    exp = OracleRegex(re).find_iter(text)
    dev = torch.from_numpy(np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    counts, m = re.find_iter_batch(dev, stride=len(text), length=len(text), count=1, capacity=17)
    assert int(counts[0]) == len(exp)
    assert [tuple(map(int, x)) for x in m.cpu().numpy()] == exp[:17]
    counts, m = re.find_iter_batch(dev, stride=len(text), length=len(text), count=1)
    assert [tuple(map(int, x)) for x in m.cpu().numpy()] == exp


def test_empty_batches_and_inputs(cuda):
    import torch
    re = R.Regex(r"a")
    dev = torch.zeros(16, dtype=torch.uint8, device=cuda)
    assert re.find_batch(dev, stride=4, length=4, count=0).shape == (0, 2)
    counts, m = re.find_iter_batch(dev, stride=4, length=4, count=0)
    assert counts.numel() == 0 and m.shape[0] == 0
    assert re.find(b"") is None and not re.is_match(b"")
    assert R.Regex(r"").find(b"") == (0, 0)
    assert R.Regex(r"").find_iter(b"") == [(0, 0)]
    rs = R.RegexSet([r"a", r"^$"])
    assert rs.matches(b"") == [1]
