"""Small batches of medium haystacks (BASELINE C1's shape, 1024 x 1 KiB) are
split into units of >= 128 B scanned with the cut-bounded search
(dispatch.cpp long_batch, long_scan_kernel) instead of one lane per haystack.
is_match takes it (find / shortest_match units would scan on until the DFA
dies: a never-dying pattern costs every unit the rest of its haystack);
is_match / find / shortest_match must equal the oracle and the unsplit
kernels (debug knob split=0) bit for bit, with matches crossing every unit cut,
Unicode and invalid UTF-8 bytes, start > 0 and ragged strides."""
import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex
from unicode_mix import unicode_mix

pytestmark = pytest.mark.gpu

# DFA without a quit state (no Unicode \b), not end-anchored: these take the split
SPLIT_PATS = [r"\d{4}-\d{2}-\d{2}", r"\w+@\w+\.\w+", r"(?m)^abc$", r"(a|ab)(c|bcd)", r"x*"]
PATS = [r"\d{4}-\d{2}-\d{2}", r"\w+@\w+\.\w+", r"(?m)^abc$", r"\bfoo\b", r"a[^x]{20,200}b", r"(a|ab)(c|bcd)", r"x*"]


def _buf(n, L, S, seed):
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(b"0123456789-abcfoxyz@. \nAB", dtype=np.uint8)
    buf = alpha[rng.integers(0, len(alpha), size=n * S)].copy()
    unicode_mix(buf, n, S, L, seed + 1, per_hay=2, frac=0.5)
    return buf


@pytest.mark.parametrize("pat", PATS)
@pytest.mark.parametrize("shape", [(1024, 1024, 1024), (300, 1000, 1008), (64, 5000, 5008)])
def test_split_small_batch(cuda, knobs, pat, shape):
    import torch
    n, L, S = shape
    buf = _buf(n, L, S, 0x5151 + n)
    d = torch.from_numpy(buf).to(cuda)
    re = R.Regex(pat)
    o = OracleRegex(re)
    for start in (0, 7):
        got_f = re.find_batch(d, stride=S, length=L, count=n, start=start).cpu().numpy()
        got_s = re.shortest_match_batch(d, stride=S, length=L, count=n, start=start).cpu().numpy()
        got_m = re.is_match_batch(d, stride=S, length=L, count=n, start=start).cpu().numpy()
        if pat in SPLIT_PATS:  # only is_match takes the split (a find unit scans until the DFA dies)
            assert N.rure_amd_last_fwd_path() == -4, (pat, shape)
        knobs(split=0)
        ref_f = re.find_batch(d, stride=S, length=L, count=n, start=start).cpu().numpy()
        ref_m = re.is_match_batch(d, stride=S, length=L, count=n, start=start).cpu().numpy()
        ref_s = re.shortest_match_batch(d, stride=S, length=L, count=n, start=start).cpu().numpy()
        knobs()
        assert np.array_equal(got_f, ref_f), (pat, shape, start)
        assert np.array_equal(got_m, ref_m), (pat, shape, start)
        assert np.array_equal(got_s, ref_s), (pat, shape, start)
        for i in range(0, n, max(1, n // 97)):
            h = bytes(buf[i * S: i * S + L])
            e = o.find(h, start)
            g = None if got_f[i, 0] < 0 else (int(got_f[i, 0]), int(got_f[i, 1]))
            assert g == e, (pat, shape, start, i)
            assert bool(got_m[i]) == o.is_match(h, start)
