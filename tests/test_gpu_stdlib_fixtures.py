"""The GPU kernels against Python's `re` answers for the BASELINE patterns
(tests/golden/stdlib_re_fixtures.json.gz): the set kernel for the 64 C4
patterns, the tile / per-lane find kernels for the date regex and find /
find_iter for the email regex — an engine independent of the product's
compiler."""
import numpy as np
import pytest

import regex_amd as R
from golden_data import stdlib_fixtures

pytestmark = pytest.mark.gpu
FX = stdlib_fixtures()


def _ragged(hs, cuda):
    import torch
    offs = np.zeros(len(hs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(h) for h in hs])
    buf = np.frombuffer(b"".join(hs) + b"\0" * 16, dtype=np.uint8).copy()
    return torch.from_numpy(buf).to(cuda), torch.from_numpy(offs).to(cuda)


def test_c4_set_kernel_vs_stdlib(cuda):
    c4 = FX["c4"]
    lines = [l.encode() for l in c4["lines"]]
    hay, offs = _ragged(lines, cuda)
    rs = R.RegexSet(c4["patterns"])
    got = rs.matches_batch(hay, offsets=offs).cpu().numpy().view(np.uint64)
    for i, exp in enumerate(c4["matches"]):
        assert [j for j in range(64) if (int(got[i]) >> j) & 1] == exp, c4["lines"][i]


def test_date_tile_kernel_vs_stdlib(cuda):
    import torch
    d = FX["date"]
    hs = [h.encode() for h in d["haystacks"]]
    L = 200
    S = 208  # 16-byte stride: the coalesced-tile kernel
    buf = np.zeros(len(hs) * S, dtype=np.uint8)
    for i, h in enumerate(hs):
        buf[i * S:i * S + L] = np.frombuffer(h, dtype=np.uint8)
    re = R.Regex(d["pattern"])
    got = re.find_batch(torch.from_numpy(buf).to(cuda), stride=S, length=L, count=len(hs)).cpu().numpy()
    hay, offs = _ragged(hs, cuda)
    got2 = re.find_batch(hay, offsets=offs).cpu().numpy()
    for i, exp in enumerate(d["find"]):
        e = tuple(exp) if exp else (-1, -1)
        assert tuple(int(x) for x in got[i]) == e and tuple(int(x) for x in got2[i]) == e, d["haystacks"][i]


def test_email_vs_stdlib(cuda):
    d = FX["email"]
    hs = [h.encode() for h in d["haystacks"]]
    hay, offs = _ragged(hs, cuda)
    re = R.Regex(d["pattern"])
    got = re.find_batch(hay, offsets=offs).cpu().numpy()
    counts, m = re.find_iter_batch(hay, offsets=offs)
    recs = [(int(a), int(b)) for a, b in m.cpu().numpy()]
    k = 0
    for i, (exp, expi) in enumerate(zip(d["find"], d["find_iter"])):
        assert tuple(int(x) for x in got[i]) == (tuple(exp) if exp else (-1, -1)), d["haystacks"][i]
        assert recs[k:k + int(counts[i])] == [tuple(x) for x in expi], d["haystacks"][i]
        k += int(counts[i])
