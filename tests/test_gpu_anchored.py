"""DfaAnchoredReverse on the GPU (dfa_anchored_rev_kernel): regexes anchored
at the end and not at the start run the reverse DFA from each haystack's end
(exec.rs:671-688, 1175-1177).  Batched find / is_match / shortest_match /
captures / find_iter against the oracle, with search starts > 0 (where the
reverse DFA's view of text[start..] differs from the forward look-behind),
Unicode word boundaries that quit the DFA (Pike VM fallback), and the C4
end-anchored patterns over log lines."""
import zlib

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex
from regex_amd.workloads import date_haystacks_host, log_lines_host

pytestmark = pytest.mark.gpu

PATTERNS = [r"\d$", r"ms$", r"s$", r"Z$", r"(?-u)\bx$", r"(?m)^x\z", r"\bfoo$", r"x*$", r"$", r"(a|ab)$",
            r"[a-z]+$", r"\d{4}-\d{2}-\d{2}$", r"(?-u)\b\w+\z"]


def _texts(n, seed):
    rng = np.random.default_rng(seed)
    alpha = [b"a", b"b", b"x", b"s", b"m", b"Z", b"1", b"9", b" ", b"\n", b"-", b"foo", "é".encode(), b"\xff"]
    out = []
    for i in range(n):
        k = int(rng.integers(0, 40))
        out.append(b"".join(alpha[int(j)] for j in rng.integers(0, len(alpha), size=k)))
    return out


def _ragged(texts, cuda):
    import torch
    offs = np.zeros(len(texts) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(t) for t in texts])
    buf = np.frombuffer(b"".join(texts) + b"\0" * 16, dtype=np.uint8).copy()
    return torch.from_numpy(buf).to(cuda), torch.from_numpy(offs).to(cuda)


@pytest.mark.parametrize("pat", PATTERNS)
@pytest.mark.parametrize("start", [0, 1, 3])
def test_anchored_reverse_batch(cuda, pat, start):
    re = R.Regex(pat)
    info, _ = re.program(2)
    assert info.anchored_end and not info.anchored_start
    o = OracleRegex(re)
    texts = _texts(3000, zlib.crc32(pat.encode()))
    hay, offs = _ragged(texts, cuda)
    got = re.find_batch(hay, offsets=offs, start=start).cpu().numpy()
    if re.uses_dfa():
        assert N.rure_amd_last_fwd_path() == -2
    ism = re.is_match_batch(hay, offsets=offs, start=start).cpu().numpy()
    sho = re.shortest_match_batch(hay, offsets=offs, start=start).cpu().numpy()
    for i, t in enumerate(texts):
        exp = o.find(t, start)
        g = None if int(got[i, 0]) == -1 else (int(got[i, 0]), int(got[i, 1]))
        assert g == exp, (pat, start, i, t, g, exp)
        assert bool(ism[i]) == o.is_match(t, start), (pat, start, t)
        es = o.shortest_match(t, start)
        assert (None if int(sho[i]) == -1 else int(sho[i])) == es, (pat, start, t)


@pytest.mark.parametrize("pat", [r"\d$", r"(?-u)\bx$", r"x*$", r"$", r"(a|ab)$"])
@pytest.mark.parametrize("start", [0, 2])
def test_anchored_reverse_find_iter(cuda, pat, start):
    re = R.Regex(pat)
    o = OracleRegex(re)
    texts = _texts(500, 7 + start)
    hay, offs = _ragged(texts, cuda)
    counts, m = re.find_iter_batch(hay, offsets=offs, start=start)
    got = [(int(a), int(b)) for a, b in m.cpu().numpy()]
    k = 0
    for i, t in enumerate(texts):
        exp = o.find_iter(t, start)
        assert int(counts[i]) == len(exp), (pat, i, t)
        assert got[k:k + len(exp)] == exp, (pat, i, t)
        k += len(exp)


def test_anchored_reverse_captures(cuda):
    re = R.Regex(r"(?-u)\b(\w)(\w*)$")
    o = OracleRegex(re)
    texts = [b"ab cd", b"x", b"", b"a b!", b"word"]
    hay, offs = _ragged(texts, cuda)
    for start in (0, 1, 3):
        got = re.captures_batch(hay, offsets=offs, start=start).cpu().numpy()
        for i, t in enumerate(texts):
            exp = o.captures(t, start)
            g = None if got[i, 0, 0] == -1 else [None if a == -1 else (int(a), int(b)) for a, b in got[i]]
            assert g == exp, (start, t, g, exp)


def test_anchored_reverse_c4_patterns(cuda):
    """The C4 set's end-anchored members searched one by one over log lines."""
    import torch
    buf, offs = log_lines_host(20000, seed=11)
    hay = torch.from_numpy(np.concatenate([buf, np.zeros(16, dtype=np.uint8)])).to(cuda)
    od = torch.from_numpy(offs).to(cuda)
    for pat in (r"ms$", r"s$", r"Z$"):
        re = R.Regex(pat)
        o = OracleRegex(re)
        got = re.find_batch(hay, offsets=od).cpu().numpy()
        exp, _ = o.find_batch(buf, 0, 0, 20000, nthreads=8, offsets=offs.astype(np.uint64))
        assert np.array_equal(got, exp.astype(np.int64)), pat


def test_anchored_reverse_strided_dates(cuda):
    import torch
    n, L = 8192, 256
    buf, _ = date_haystacks_host(n, L, seed=3, frac=0.0)
    for i in range(0, n, 3):  # dates ending every third haystack
        buf[i * L + L - 10:(i + 1) * L] = np.frombuffer(b"2017-12-30", dtype=np.uint8)
    re = R.Regex(r"\d{4}-\d{2}-\d{2}$")
    o = OracleRegex(re)
    got = re.find_batch(torch.from_numpy(buf).to(cuda), stride=L, length=L, count=n).cpu().numpy()
    exp, _ = o.find_batch(buf, L, L, n, nthreads=8)
    assert np.array_equal(got, exp.astype(np.int64))
    assert (got[:, 0] >= 0).sum() >= n // 3
