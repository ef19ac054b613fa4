"""The find_iter run engine on the GPU (run_iter.hip, last_fwd_path -19):
C+ regexes' matches = maximal runs, against the oracle's find_iter
(re_trait.rs:197-221) — single long haystacks (runs crossing lanes and 4 KiB
units, a run longer than many units, all-C text), fixed-stride batches,
searches from start > 0, and text with bytes >= 0x80 (a Unicode class reads
them as UTF-8, valid or not, and still answers)."""
import gzip
import os
import random
import zlib

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PATS = [r"\w+", r"[a-z]+", r"\S+", r"\pL+", r"\d+", r"(?-u)\w+", r"[^\n]+", r"\s+", r"(?i)[a-f]+"]


def sherlock():
    return gzip.open(os.path.join(HERE, "golden", "sherlock.txt.gz")).read()


def dev(t, cuda):
    import torch
    a = np.frombuffer(t, dtype=np.uint8)
    return torch.from_numpy(np.concatenate([a, np.zeros(16, np.uint8)])).to(cuda)


def check_one(re, t, cuda, start=0, expect_path=None):
    counts, m = re.find_iter_batch(dev(t, cuda), stride=len(t), length=len(t), count=1, start=start)
    got = [tuple(x) for x in m.cpu().numpy().tolist()]
    exp = OracleRegex(re).find_iter(t, start)
    assert int(counts[0]) == len(exp)
    assert got == exp
    if expect_path is not None:
        assert N.rure_amd_last_fwd_path() == expect_path


@pytest.mark.parametrize("pat", PATS)
def test_runs_sherlock(cuda, pat):
    t = sherlock()
    t = bytes(b if b < 0x80 else 0x20 for b in t)  # ASCII: the run engine answers
    re = R.Regex(pat)
    check_one(re, t, cuda, expect_path=-19)
    check_one(re, t, cuda, start=4097)


@pytest.mark.parametrize("pat", [r"\w+", r"[a-z]+", r"[^\n]+"])
def test_runs_long_and_all_c(cuda, pat):
    re = R.Regex(pat)
    rng = random.Random(7)
    # runs crossing lanes (64 B) and units (4 KiB), one far longer than a unit
    parts = []
    for i in range(300):
        parts.append(b"a" * rng.choice([1, 63, 64, 65, 4095, 4096, 4097, 9000]))
        parts.append(b" " * rng.choice([1, 2, 64]))
    parts.append(b"b" * 100000)
    t = b"".join(parts)
    check_one(re, t, cuda, expect_path=-19)
    check_one(re, b"z" * 70000, cuda)  # one run: the whole text
    check_one(re, b"z" * 8192, cuda)   # ... ending exactly at a unit edge
    check_one(re, b"", cuda)


@pytest.mark.parametrize("pat", [r"\w+", r"(?-u)\w+"])
def test_runs_stride_batch(cuda, pat):
    import torch
    re = R.Regex(pat)
    t = sherlock()
    t = bytes(b if b < 0x80 else 0x2e for b in t)
    L, n = 5008, 40  # 16-byte stride
    hay = np.frombuffer(t[: L * n], dtype=np.uint8)
    d = torch.from_numpy(np.concatenate([hay, np.zeros(16, np.uint8)])).to(cuda)
    for start in (0, 16, 3):
        counts, m = re.find_iter_batch(d, stride=L, length=L - 8, count=n, start=start)
        got = [tuple(x) for x in m.cpu().numpy().tolist()]
        o = OracleRegex(re)
        exp = []
        for i in range(n):
            e = o.find_iter(t[i * L:i * L + L - 8], start)
            assert int(counts[i]) == len(e)
            exp += e
        assert got == exp, (pat, start)


@pytest.mark.parametrize("pat", [r"\w+", r"\S+", r"\pL+", r"[a-z]+", r"\d+", r"(?i)[a-z]+", r"[^\n]+", r".+"])
def test_runs_non_ascii(cuda, pat):
    """Bytes >= 0x80: a Unicode class's engine decodes them as UTF-8 (valid
    letters, marks, digits, symbols, astral code points; stray
    continuations, truncated leads, overlong forms, surrogates, bytes past
    U+10FFFF) and still answers (-19), with runs crossing lanes and units;
    [a-z]+'s class is exact on every byte."""
    from test_run_engine import utf8_text
    re = R.Regex(pat)
    rng = random.Random(3)
    alpha = [b"ab", b"Z9", b" ", b"\n", "é".encode(), "✓".encode(), b"\xff", "٣".encode(), b"x_y"]
    t = b"".join(rng.choices(alpha, k=30000))
    check_one(re, t, cuda, expect_path=-19)
    check_one(re, t, cuda, start=4097)
    u = utf8_text(zlib.crc32(pat.encode()), 40000)
    check_one(re, u, cuda, expect_path=-19)
    for st in (1, 2, 63, 4095, 4097):
        check_one(re, u, cuda, start=st)
    # a multi-byte encoding straddling every lane and unit edge: é at 62-63,
    # 中 at 4094-4096, an astral letter at 8190-8193
    edge = bytearray(b"a" * 12288)
    edge[62:64] = "é".encode()
    edge[4094:4097] = "中".encode()
    edge[8190:8194] = "\U0001d400".encode()
    edge[200:201] = b" "
    check_one(re, bytes(edge), cuda, expect_path=-19)


def test_runs_sherlock_unicode(cuda):
    r"""The sherlock corpus as it is (with its non-ASCII bytes): \w+ = the
    reference's count 109214 (bench/src/sherlock.rs:116) on the run engine."""
    re = R.Regex(r"\w+")
    t = sherlock()
    assert any(b >= 0x80 for b in t)
    check_one(re, t, cuda, expect_path=-19)
    counts, _ = re.find_iter_batch(dev(t, cuda), stride=len(t), length=len(t), count=1)
    assert int(counts[0]) == 109214
