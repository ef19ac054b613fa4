"""RegexSet of more than 64 patterns on the GPU (rure_amd_set_matches_batch_words
and rure_set_matches) against the oracle over the combined set program."""
import numpy as np
import pytest

import regex_amd as R
from bigset_data import SETS
from oracle_py import OracleRegex
from regex_amd.workloads import log_lines_host

pytestmark = pytest.mark.gpu


def _bits(row, k):
    return [j for j in range(k) if (int(row[j // 64]) >> (j % 64)) & 1]


@pytest.mark.parametrize("k", sorted(SETS))
def test_big_set_batch(cuda, k):
    import torch
    rs = R.RegexSet(SETS[k])
    o = OracleRegex(rs)
    buf, offs = log_lines_host(3000, seed=0xB16 + k)
    buf = np.concatenate([buf, np.zeros(16, dtype=np.uint8)])
    got = rs.matches_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy()
    assert got.shape == (3000, rs.words)
    for i in range(3000):
        t = bytes(buf[offs[i]:offs[i + 1]])
        exp = o.matches(t)
        assert _bits(got[i].view(np.uint64), k) == exp, (k, i)
        if i % 97 == 0:
            assert rs.matches(t) == exp
            assert rs.is_match(t) == bool(exp)


def test_big_set_strided_and_start(cuda):
    import torch
    k = 100
    rs = R.RegexSet(SETS[k])
    o = OracleRegex(rs)
    n, L = 500, 160
    buf, offs = log_lines_host(n, seed=5, lo=L, hi=L)
    dev = torch.from_numpy(np.concatenate([buf, np.zeros(16, dtype=np.uint8)])).to(cuda)
    for start in (0, 7):
        got = rs.matches_batch(dev, stride=L, length=L, count=n, start=start).cpu().numpy()
        for i in range(n):
            t = bytes(buf[i * L:(i + 1) * L])
            assert _bits(got[i].view(np.uint64), k) == o.matches(t, start), (start, i)


def test_small_sets_words_api(cuda):
    """The words entry point also serves sets of 0, 1 and <= 64 patterns."""
    import ctypes
    import torch
    from regex_amd import _native as N
    texts = [b"foo", b"bar", b"", b"xfoo"]
    L = 8
    buf = np.zeros(len(texts) * L + 16, dtype=np.uint8)
    for i, t in enumerate(texts):
        buf[i * L:i * L + len(t)] = np.frombuffer(t, dtype=np.uint8) if t else []
    dev = torch.from_numpy(buf).to(cuda)
    lens = torch.tensor([len(t) for t in texts])
    offs = torch.zeros(len(texts) + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(lens, 0)
    # ragged offsets over the packed texts
    packed = np.frombuffer(b"".join(texts) + bytes(16), dtype=np.uint8).copy()
    pd = torch.from_numpy(packed).to(cuda)
    for pats in ([], ["foo"], ["foo", "^x", "r$"]):
        rs = R.RegexSet(pats)
        out = torch.full((len(texts), 2), -5, dtype=torch.int64, device=cuda)
        b = R._batch(pd, offs.to(cuda))
        rc = N.rure_amd_set_matches_batch_words(rs._set, ctypes.byref(b), ctypes.c_void_p(out.data_ptr()), 2,
                                                R._stream_ptr(None))
        assert rc == N.OK
        got = out.cpu().numpy()
        for i, t in enumerate(texts):
            assert _bits(got[i].view(np.uint64), len(pats)) == rs.matches(t), (pats, t)
            assert got[i, 1] == 0
