"""The line-stream set kernel (`set_stream_kernel`): offset
batches of many lines, each lane streaming a run of lines as aligned blocks.
Bit-exact against the oracle's DfaMany restatement (exec.rs:998-1038,
dfa.rs:525-570) per line, at the natural dispatch size (>= 4 lines per lane
of the full grid) and forced (RURE_AMD_SET_STREAM=1) on ragged batches that
reach every path: line ends inside a block, blocks holding several line
ends (lines < 16 bytes, empty lines), waves of short lines (one line per
lane), steps that leave the hot cores (a small LDS budget), quits (Unicode
\\b over non-ASCII bytes)."""
import numpy as np
import pytest

import regex_amd as R
from oracle_py import OracleRegex
from regex_amd.workloads import C4_PATTERNS, log_lines_host

pytestmark = pytest.mark.gpu


def _check(rs, buf, offs, cuda, nthreads=16):
    import torch
    n = len(offs) - 1
    dev = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(cuda)
    got = rs.matches_batch(dev, offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy().astype(np.uint64)
    exp = OracleRegex(rs).set_batch(buf, 0, 0, n, nthreads=nthreads, offsets=offs)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (bad[:10], got[bad[:10]], exp[bad[:10]])


def _recut(buf, lens):
    """Offsets cutting buf (repeated as needed) into lines of the given lengths."""
    total = int(lens.sum())
    reps = total // len(buf) + 1
    b = np.tile(buf, reps)[:total].copy()
    offs = np.zeros(len(lens) + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    return b, offs


def test_c4_stream_natural(cuda, monkeypatch):
    """C4's lines, 1.1 M of them (> 4 lines per lane of the full grid)."""
    from regex_amd import _native as N
    monkeypatch.setenv("RURE_AMD_SET_STREAM", "1")
    n = 1_100_000
    buf, offs = log_lines_host(n, seed=0x5EED0004)
    rs = R.RegexSet(C4_PATTERNS)
    _check(rs, buf, offs, cuda)
    assert N.rure_amd_last_fwd_path() == -18


@pytest.mark.parametrize("kind", ["mixed", "short", "long", "huge", "empty_runs"])
def test_stream_ragged_forced(cuda, monkeypatch, kind):
    monkeypatch.setenv("RURE_AMD_SET_STREAM", "1")
    rng = np.random.default_rng(hash(kind) & 0xFFFF)
    base, _ = log_lines_host(20000, seed=7)
    if kind == "mixed":      # empty lines, lines < 16 bytes and long ones
        lens = rng.choice([0, 1, 3, 15, 16, 17, 31, 64, 100, 161, 700], size=60000)
    elif kind == "short":    # waves of short lines: one line per lane
        lens = rng.integers(0, 24, size=80000)
    elif kind == "long":
        lens = rng.integers(200, 5000, size=4000)
    elif kind == "huge":     # a few lines far longer than a lane's share
        lens = np.array([0, 1 << 20, 5, 300000, 17, 1 << 19, 0, 0, 99], dtype=np.int64)
    else:                    # runs of empty lines between C4-like lines
        lens = np.where(rng.random(50000) < 0.3, 0, rng.integers(40, 160, size=50000))
    buf, offs = _recut(base, lens.astype(np.int64))
    rs = R.RegexSet(C4_PATTERNS)
    _check(rs, buf, offs, cuda)


def test_stream_non_ascii_quit(cuda, monkeypatch):
    """Unicode \\b members quit on non-ASCII bytes: QUITMARK lines go to the
    Pike VM pass, the others keep the stream kernel's masks."""
    monkeypatch.setenv("RURE_AMD_SET_STREAM", "1")
    n = 30000
    buf, offs = log_lines_host(n, seed=99)
    buf = buf.copy()
    rng = np.random.default_rng(5)
    pos = rng.integers(0, len(buf), size=n // 5)
    buf[pos] = rng.choice(np.frombuffer("é✓".encode(), dtype=np.uint8), size=len(pos))
    rs = R.RegexSet(C4_PATTERNS)
    _check(rs, buf, offs, cuda)


def test_stream_small_hot_set(cuda, monkeypatch):
    """A small LDS budget: many steps leave the hot cores (careful path with
    the global tables), still bit-exact."""
    monkeypatch.setenv("RURE_AMD_SET_STREAM", "1")
    monkeypatch.setenv("RURE_AMD_CORE_LDS", "12000")
    n = 20000
    buf, offs = log_lines_host(n, seed=3)
    rs = R.RegexSet(C4_PATTERNS)
    _check(rs, buf, offs, cuda)


def test_stream_sherlock_lines(cuda, monkeypatch):
    """Real text lines (many short and empty ones) with word-class patterns."""
    import gzip
    import os
    monkeypatch.setenv("RURE_AMD_SET_STREAM", "1")
    here = os.path.dirname(os.path.abspath(__file__))
    text = gzip.open(os.path.join(here, "golden", "sherlock.txt.gz")).read()
    lines = text.split(b"\n")
    buf = np.frombuffer(b"".join(lines), dtype=np.uint8).copy()
    offs = np.zeros(len(lines) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(x) for x in lines])
    pats = [r"Holmes", r"\bWatson\b", r"\w+ing\b", r"(?i)sherlock", r"[A-Z][a-z]+\s+[A-Z]", r"^The", r"\d+",
            r"\.$", r"(?m)^$", r"\bthe\b", r"[aeiou]{3}", r"\w{12,}", r"[,;:]\s", r"'s\b", r"\bI\b", r"said"]
    rs = R.RegexSet(pats)
    _check(rs, buf, offs, cuda)
