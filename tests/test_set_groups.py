"""Sets of more than 64 patterns on the CPU: the grouped evaluation the GPU
uses (64 consecutive patterns per group, runtime.hpp rure_set::groups) gives
the combined set's answer.  Checked with the oracle (restated DfaMany /
Pike VM, dfa.rs:525-570, pikevm.rs:150-180) over the combined program versus
the oracle over each group's own program, on log lines and odd haystacks."""
import pytest

import regex_amd as R
from bigset_data import SETS
from oracle_py import OracleRegex
from regex_amd.workloads import log_lines_host

TEXTS = [b"", b"nil", b"s", b"ok", b"killed", b"\xff\xfe INFO x ERROR", "ün ERROR über".encode(),
         b"GET /api/v1/items HTTP/1.1 status=404 latency=123ms", b"  ", b"aio quu zz"]


@pytest.mark.parametrize("k", sorted(SETS))
def test_groups_equal_combined(k):
    pats = SETS[k]
    rs = R.RegexSet(pats)
    assert len(rs) == k and rs.words == (k + 63) // 64
    whole = OracleRegex(rs)
    groups = [(lo, OracleRegex(R.RegexSet(pats[lo:lo + 64])) if len(pats[lo:lo + 64]) > 1
               else OracleRegex(R.Regex(pats[lo]))) for lo in range(0, k, 64)]
    buf, offs = log_lines_host(400, seed=k)
    texts = TEXTS + [bytes(buf[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]
    for t in texts:
        exp = whole.matches(t)
        got = []
        for lo, o in groups:
            if hasattr(o, "n"):
                got += [lo + j for j in o.matches(t)]
            elif o.is_match(t):
                got.append(lo)
        assert got == exp, (k, t)


def test_big_set_compile():
    """Compile-time behaviour of a large set (no GPU): length, program export
    of the combined set, the error for an invalid member."""
    rs = R.RegexSet(SETS[100])
    info, _ = rs.program(0)
    assert info.nmatches == 100
    with pytest.raises(R.Error):
        R.RegexSet(SETS[100] + ["(unclosed"])
