"""Ragged (offset) batches of one regex on dfa_line_kernel (dfa_scan.hip):
find / is_match / shortest_match per line against the oracle (the restated
lazy DFA, dfa.rs:576-764, and exec.rs:632-662 / 382-420 dispatch).

Lines of every shape the kernel's masked head / tail blocks and its
one-line-ahead prefetch meet: empty lines, 1-byte lines, lines inside one
16-byte block, lines crossing many blocks, lines > 4 KiB, runs of empty lines
at the end of the batch, lines carrying Unicode digits / word characters and
invalid UTF-8 (the sentinel redo on the global table), and searches from
start > 0 (look-behind from the byte before start).  rure_amd_last_fwd_path()
== -8 asserts the line kernel ran; debug knob lines=0 gives the previous
one-lane-per-haystack kernel, checked for the same answers.
"""
import os

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex
from regex_amd.workloads import date_haystacks_host
from unicode_mix import unicode_mix

pytestmark = pytest.mark.gpu

PATS = [r"\d{4}-\d{2}-\d{2}", r"\w+@\w+\.\w+", r"Sherlock\s+\w+", r"(?m)^\d+$", r"\bfox\b", r"[a-z]+ing\b",
        r"x*", r"(?-u)\xFF+"]


def _lines(n, seed, maxlen=300, long_every=0):
    rng = np.random.default_rng(seed)
    kind = rng.integers(0, 10, size=n)
    lens = np.where(kind == 0, 0, np.where(kind == 1, 1, np.where(kind == 2, rng.integers(2, 16, size=n),
                                                                  rng.integers(16, maxlen, size=n))))
    if long_every:
        lens[::long_every] = rng.integers(4097, 9000, size=lens[::long_every].size)
    lens[-5:] = 0  # empty lines at the end of the batch
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    total = int(offs[-1])
    buf, _ = date_haystacks_host(1, total + 64, seed=seed ^ 0x33, frac=0.0)
    # dates, words, emails and Unicode planted per 64-byte window
    unicode_mix(buf, len(buf) // 64, 64, 64, seed ^ 0x5A, per_hay=1, frac=0.4)
    words = [b"Sherlock Holmes", b"ann@example.org", b"2017-12-30", b"running", b"fox", b"1234\n", b"\xff\xff"]
    for i in rng.integers(0, max(1, total - 20), size=max(1, total // 80)):
        w = words[int(rng.integers(len(words)))]
        buf[i:i + len(w)] = np.frombuffer(w, dtype=np.uint8)
    return buf, offs


def _check(cuda, re, o, buf, offs, start):
    import torch
    n = offs.size - 1
    d = torch.from_numpy(buf).to(cuda)
    od = torch.from_numpy(offs).to(cuda)
    got = re.find_batch(d, offsets=od, start=start).cpu().numpy()
    path = N.rure_amd_last_fwd_path()
    ism = re.is_match_batch(d, offsets=od, start=start).cpu().numpy()
    sho = re.shortest_match_batch(d, offsets=od, start=start).cpu().numpy()
    if start == 0:
        exp, _ = o.find_batch(buf, 0, 0, n, nthreads=8, offsets=offs.astype(np.uint64))
        exp = exp.astype(np.int64)
        iexp = o.is_match_batch(buf, 0, 0, n, nthreads=8, offsets=offs.astype(np.uint64)).astype(bool)
        sexp = o.shortest_batch(buf, 0, 0, n, nthreads=8, offsets=offs.astype(np.uint64)).astype(np.int64)
    else:
        exp = np.full((n, 2), -1, dtype=np.int64)
        iexp = np.zeros(n, dtype=bool)
        sexp = np.full(n, -1, dtype=np.int64)
        for i in range(n):
            h = bytes(buf[offs[i]:offs[i + 1]])
            m = o.find(h, start)
            if m is not None:
                exp[i] = m
            iexp[i] = o.is_match(h, start)
            s = o.shortest_match(h, start)
            if s is not None:
                sexp[i] = s
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert bad.size == 0, (re.pattern, start, int(bad[0]), got[bad[0]].tolist(), exp[bad[0]].tolist())
    assert np.array_equal(ism.astype(bool), iexp), re.pattern
    sbad = np.nonzero(sho.astype(np.int64) != sexp)[0]
    assert sbad.size == 0, (re.pattern, start, int(sbad[0]), int(sho[sbad[0]]), int(sexp[sbad[0]]))
    return path, got


@pytest.mark.parametrize("pat", PATS)
def test_lines_parity(cuda, pat):
    re = R.Regex(pat)
    o = OracleRegex(re)
    buf, offs = _lines(30_000, 0x11 + len(pat))
    path, got = _check(cuda, re, o, buf, offs, 0)
    # the previous per-lane kernel gives the same answers (A/B switch)
    import torch
    with R.debug(lines=0):
        got0 = re.find_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy()
    assert np.array_equal(got, got0)


def test_lines_path_taken(cuda):
    re = R.Regex(r"\d{4}-\d{2}-\d{2}")
    o = OracleRegex(re)
    buf, offs = _lines(5000, 7)
    path, _ = _check(cuda, re, o, buf, offs, 0)
    assert path == -8


@pytest.mark.parametrize("pat", [r"\d{4}-\d{2}-\d{2}", r"\bfox\b", r"(?m)^\d+$"])
def test_lines_long(cuda, pat):
    """lines > 4 KiB between short ones (a wave's lanes diverge by 1000x)"""
    re = R.Regex(pat)
    o = OracleRegex(re)
    buf, offs = _lines(3000, 0x77, long_every=37)
    _check(cuda, re, o, buf, offs, 0)


@pytest.mark.parametrize("start", [1, 5, 17])
def test_lines_start(cuda, start):
    """search from start > 0 (look-behind from text[start - 1], dfa.rs:1415-1434;
    lines shorter than start have no match)"""
    for pat in (r"\d{4}-\d{2}-\d{2}", r"\bfox\b", r"(?m)^\d+$", r"x*"):
        re = R.Regex(pat)
        o = OracleRegex(re)
        buf, offs = _lines(1500, 0x99 + start, maxlen=60)
        _check(cuda, re, o, buf, offs, start)


def test_lines_tiny_batches(cuda):
    """batches of 1, 2 and 65 lines (a partial wave, the clamped prefetch)"""
    re = R.Regex(r"\w+@\w+\.\w+")
    o = OracleRegex(re)
    for n in (1, 2, 65):
        buf, offs = _lines(n + 5, 0x42 + n)
        _check(cuda, re, o, buf, offs[: n + 1].copy(), 0)
