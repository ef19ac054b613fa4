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


@pytest.mark.parametrize("where", ["late", "early", "none"])
def test_long_shard_4gib(cuda, where):
    """C5's shape past 2^32 bytes (one 4.5 GiB haystack, 64-bit offsets, the
    chunked long scan): synthetic text without '@', addresses planted at
    known places; find / is_match / shortest_match must report the first
    (size-independent: the answer is known without scanning on the CPU).
    The oracle checks the same planting on a 1 MiB window around it."""
    import torch
    L = (9 << 29) + 12345  # 4.5 GiB + a ragged tail
    g = torch.Generator(device=cuda).manual_seed(0xC5)
    # printable ASCII without '@' (0x40): 0x20..0x3F and 0x41..0x7E, word
    # bytes separated often enough that \w+ runs stay short
    t = torch.randint(0, 94, (L + 16,), dtype=torch.uint8, device=cuda, generator=g)
    t += 0x20
    t += (t >= 0x40).to(torch.uint8)  # elementwise (masked indexing overflows at this size)
    t[L:] = 0
    plants = {"late": [L - 777, L - 5_000_000], "early": [3_000_000_123, (1 << 32) + 99], "none": []}[where]
    addr = torch.tensor(list(b" me@host.org "), dtype=torch.uint8, device=cuda)
    for p in plants:
        t[p:p + 13] = addr
    re = R.Regex(r"\w+@\w+\.\w+")
    got = re.find_batch(t, stride=L, length=L, count=1).cpu().numpy()[0]
    first = min(plants) if plants else None
    exp = (first + 1, first + 12) if plants else None
    assert (None if got[0] < 0 else (int(got[0]), int(got[1]))) == exp
    ism = re.is_match_batch(t, stride=L, length=L, count=1).cpu().numpy()[0]
    assert bool(ism) == bool(plants)
    sho = int(re.shortest_match_batch(t, stride=L, length=L, count=1).cpu().numpy()[0])
    if not plants:
        assert sho < 0
        return
    # the oracle on a window around the first planting (nothing before it
    # can match: the text has no '@') gives the same find and shortest end
    lo = max(0, first - (1 << 19))
    win = bytes(t[lo:lo + (1 << 20)].cpu().numpy())
    o = OracleRegex(re)
    s, e = o.find(win)
    assert (lo + s, lo + e) == exp
    assert sho == lo + o.shortest_match(win)
