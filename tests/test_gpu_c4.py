"""C4 shape (BASELINE.json configs[3]): the 64-pattern RegexSet over
synthetic log lines, GPU set kernel vs the oracle (forward_many / Pike VM
dispatch of exec.rs:998-1038), bit-exact per line."""
import numpy as np
import pytest

import regex_amd as R
from oracle_py import OracleRegex
from regex_amd.workloads import C4_PATTERNS, log_lines_host

pytestmark = pytest.mark.gpu


def test_c4_set_lines(cuda):
    import torch
    n = 20000
    buf, offs = log_lines_host(n)
    rs = R.RegexSet(C4_PATTERNS)
    assert rs.uses_dfa()
    got = rs.matches_batch(torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(cuda),
                           offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy().astype(np.uint64)
    exp = OracleRegex(rs).set_batch(buf, 0, 0, n, nthreads=8, offsets=offs)
    assert np.array_equal(got, exp)


def test_c4_set_lines_non_ascii(cuda):
    """Unicode word boundaries in the set: lines with non-ASCII bytes take the
    Pike VM fallback."""
    import torch
    n = 3000
    buf, offs = log_lines_host(n, seed=99)
    buf = buf.copy()
    rng = np.random.default_rng(5)
    pos = rng.integers(0, len(buf), size=n // 3)
    buf[pos] = rng.choice(np.frombuffer("é✓".encode(), dtype=np.uint8), size=len(pos))
    rs = R.RegexSet(C4_PATTERNS)
    got = rs.matches_batch(torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(cuda),
                           offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy().astype(np.uint64)
    exp = OracleRegex(rs).set_batch(buf, 0, 0, n, nthreads=8, offsets=offs)
    assert np.array_equal(got, exp)


def _mixed_lines(n, seed):
    """Log text cut into lines of widely mixed lengths: empty, 1-byte,
    block-sized (15/16/17), short, C4-like and multi-KiB lines, at every
    alignment (the per-lane stream kernel's head / body / tail blocks and its
    line switches)."""
    rng = np.random.default_rng(seed)
    kinds = rng.integers(0, 6, size=n)
    lens = np.select([kinds == 0, kinds == 1, kinds == 2, kinds == 3, kinds == 4],
                     [np.zeros(n, np.int64), rng.integers(1, 3, size=n), rng.integers(15, 18, size=n),
                      rng.integers(40, 161, size=n), rng.integers(161, 600, size=n)],
                     rng.integers(600, 4000, size=n))
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    src, _ = log_lines_host(int(offs[-1]) // 100 + 1, seed=seed)
    reps = int(offs[-1]) // len(src) + 1
    buf = np.tile(src, reps)[:int(offs[-1])].copy()
    return buf, offs


@pytest.mark.parametrize("kn", [{}, {"core_bs": 256}])
def test_c4_set_mixed_lengths(cuda, knobs, kn):
    """Lines of widely mixed lengths (empty to 4 KiB, every alignment)
    through the core-form set kernel, with 1024- and 256-thread blocks."""
    import torch
    n = 30000
    buf, offs = _mixed_lines(n, seed=17)
    rs = R.RegexSet(C4_PATTERNS)
    knobs(**kn)
    dev = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(cuda)
    got = rs.matches_batch(dev, offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy().astype(np.uint64)
    exp = OracleRegex(rs).set_batch(buf, 0, 0, n, nthreads=8, offsets=offs)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("n", [1, 63, 65, 1000])
@pytest.mark.parametrize("start", [0, 3, 16, 41])
def test_c4_set_mixed_lengths_start(cuda, n, start):
    """Small batches (fewer lines than lanes) with a search start: lines
    shorter than the start report nothing (the start lies past them)."""
    import torch
    buf, offs = _mixed_lines(n, seed=100 + n + start)
    rs = R.RegexSet(C4_PATTERNS)
    o = OracleRegex(rs)
    dev = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(cuda)
    got = rs.matches_batch(dev, offsets=torch.from_numpy(offs).to(cuda), start=start).cpu().numpy()
    for i in range(n):
        t = bytes(buf[offs[i]:offs[i + 1]])
        exp = sum(1 << j for j in o.matches(t, start)) if start <= len(t) else 0
        assert int(got[i]) & ((1 << 64) - 1) == exp, (i, len(t))
