"""Few long haystacks (the C5 shape, scaled down): the chunked single search
(launch_long_scan) vs the oracle, find / is_match / shortest_match."""
import numpy as np
import pytest

import regex_amd as R
from golden_data import corpus
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

PATTERNS = [r"\w+@\w+\.\w+", r"Holmes\s+\w+", r"zzzz", r"(?-u:\b)Watson(?-u:\b)", r"[A-Z][a-z]+ [A-Z]\.",
            r"(?m)^The", r"\d{4}", r"a", r"x*", r"(?s)Sherlock.{0,200}Holmes", r"w[aeiou]+\w*$"]


def haystacks(n, L, plant_at=None):
    text = corpus("sherlock")
    rep = (n * L) // len(text) + 1
    buf = np.frombuffer((text * rep)[: n * L], dtype=np.uint8).copy()
    if plant_at is not None:
        for i, pos in enumerate(plant_at):
            buf[i * L + pos:i * L + pos + 13] = np.frombuffer(b"me@host.org  ", dtype=np.uint8)
    return buf


@pytest.mark.parametrize("pat", PATTERNS)
@pytest.mark.parametrize("n", [1, 3])
def test_long_haystacks(cuda, pat, n):
    import torch
    L = 3 << 20
    buf = haystacks(n, L)
    re = R.Regex(pat)
    o = OracleRegex(re)
    dev = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(cuda)
    for start in (0, 777):
        got = re.find_batch(dev, stride=L, length=L, count=n, start=start).cpu().numpy()
        ism = re.is_match_batch(dev, stride=L, length=L, count=n, start=start).cpu().numpy()
        sho = re.shortest_match_batch(dev, stride=L, length=L, count=n, start=start).cpu().numpy()
        for i in range(n):
            t = bytes(buf[i * L:(i + 1) * L])
            exp = o.find(t, start)
            g = None if got[i, 0] < 0 else (int(got[i, 0]), int(got[i, 1]))
            assert g == exp, (pat, i, start)
            assert bool(ism[i]) == (exp is not None)
            es = o.shortest_match(t, start)
            assert (None if sho[i] < 0 else int(sho[i])) == es, (pat, i, start)


def test_long_planted_late(cuda):
    """One planted match near the end of each shard (C5's layout)."""
    import torch
    L = 8 << 20
    n = 2
    text = (b"abc def, ghi. " * ((n * L) // 14 + 1))[: n * L]
    buf = np.frombuffer(text, dtype=np.uint8).copy()
    pos = [L - 5000, L - 123456]
    for i, p in enumerate(pos):
        buf[i * L + p:i * L + p + 13] = np.frombuffer(b" me@host.org ", dtype=np.uint8)
    re = R.Regex(r"\w+@\w+\.\w+")
    dev = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(cuda)
    got = re.find_batch(dev, stride=L, length=L, count=n).cpu().numpy()
    assert [tuple(map(int, g)) for g in got] == [(p + 1, p + 12) for p in pos]
    assert re.find(bytes(buf[:L])) == (pos[0] + 1, pos[0] + 12)
