"""Parity on the exact kernels the C2 bench times (VERDICT r01 "next" 1a/1b).

The coalesced-tile kernel picks its table by batch size (dfa_scan.hip
launch_tile): batches above half the resident lanes (cus * 16 * 64 / 2 =
131,072 haystacks on MI355X) run the byte table (STRIDE = 1, the
instantiation bench.py times on 1M x 4 KiB), smaller ones the multi-byte
table when the DFA has one.  Both are compared here with the oracle (the
restated lazy DFA, dfa.rs:576-764 / exec.rs:632-662), on the printable-ASCII
date recipe and on haystacks carrying Unicode digits, multi-byte word
characters and invalid UTF-8 (the sentinel redo on the global u16 table).
rure_amd_last_fwd_path() asserts which kernel ran.
"""
import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex
from regex_amd.workloads import date_haystacks_host
from unicode_mix import unicode_mix

pytestmark = pytest.mark.gpu

DATE = r"\d{4}-\d{2}-\d{2}"
EMAIL = r"\w+@\w+\.\w+"


def _batch(n, L, seed, mix):
    buf, _ = date_haystacks_host(n, L, seed=seed, frac=0.05)
    if mix:
        unicode_mix(buf, n, L, L, seed ^ 0xA5A5, per_hay=3, frac=0.5)
    return buf


def _check(cuda, pat, n, L, seed, mix, expect_path):
    import torch
    buf = _batch(n, L, seed, mix)
    re = R.Regex(pat)
    o = OracleRegex(re)
    dev = torch.from_numpy(buf).to(cuda)
    got = re.find_batch(dev, stride=L, length=L, count=n).cpu().numpy()
    path = N.rure_amd_last_fwd_path()
    exp, _ = o.find_batch(buf, L, L, n, nthreads=8)
    exp = exp.astype(np.int64)
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert bad.size == 0, (pat, int(bad[0]), got[bad[0]].tolist(), exp[bad[0]].tolist())
    if expect_path is not None:
        assert path in expect_path, (pat, n, path)
    ism = re.is_match_batch(dev, stride=L, length=L, count=n).cpu().numpy()
    assert N.rure_amd_last_fwd_path() == path
    iexp = o.is_match_batch(buf, L, L, n, nthreads=8)
    assert np.array_equal(ism.astype(bool), iexp.astype(bool))
    sho = re.shortest_match_batch(dev, stride=L, length=L, count=n).cpu().numpy()
    # the whole batch against the oracle's shortest_match (exec.rs:382-420)
    sexp = o.shortest_batch(buf, L, L, n, nthreads=8).astype(np.int64)
    sbad = np.nonzero(sho.astype(np.int64) != sexp)[0]
    assert sbad.size == 0, (pat, int(sbad[0]), int(sho[sbad[0]]), int(sexp[sbad[0]]))
    return got


@pytest.mark.parametrize("mix", [False, True])
def test_date_byte_table_above_threshold(cuda, mix):
    """140,000 x 128 B fixed-stride haystacks: above the 131,072 threshold, so
    the STRIDE = 1 tile kernel (the C2 timed instantiation) runs."""
    got = _check(cuda, DATE, 140_000, 128, 0x7171, mix, expect_path=(1,))
    assert (got[:, 0] >= 0).sum() > 5000


@pytest.mark.parametrize("mix", [False, True])
def test_date_multibyte_table_below_threshold(cuda, mix):
    """Below the threshold the date DFA's multi-byte table runs (when built)."""
    re = R.Regex(DATE)
    fs = re.dfa_info(0)["fast_stride"]
    _check(cuda, DATE, 20_000, 256, 0x7272, mix, expect_path=(fs,))


@pytest.mark.parametrize("n", [20_000, 140_000])
def test_email_tile_unicode(cuda, n):
    _check(cuda, EMAIL, n, 128, 0x7373 + n, True, expect_path=(1, 2, 4))


def test_date_tile_long_unicode(cuda):
    """4 KiB haystacks (the C2 shape) with Unicode tokens, above the threshold."""
    _check(cuda, DATE, 132_000, 1024, 0x7474, True, expect_path=(1,))


def test_ragged_unicode(cuda):
    """The per-lane streaming kernel (ragged offsets) on the same mixes."""
    import torch
    n = 20_000
    rng = np.random.default_rng(9)
    lens = rng.integers(0, 400, size=n)
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    buf = _batch(1, int(offs[-1]) + 64, 0x7575, False)
    # plant tokens with the same generator, haystack by haystack
    unicode_mix(buf, len(buf) // 64, 64, 64, 0x7676, per_hay=1, frac=0.6)
    for pat in (DATE, EMAIL):
        re = R.Regex(pat)
        o = OracleRegex(re)
        got = re.find_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy()
        assert N.rure_amd_last_fwd_path() == -8  # dfa_line_kernel
        exp, _ = o.find_batch(buf, 0, 0, n, nthreads=8, offsets=offs.astype(np.uint64))
        assert np.array_equal(got, exp.astype(np.int64)), pat
