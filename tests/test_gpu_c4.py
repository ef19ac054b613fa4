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
