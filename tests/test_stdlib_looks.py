"""The oracle's find_iter (re_trait.rs:197-221 over exec.rs:632-662) against
Python's `re` for look-around regexes over ASCII text
(tests/golden/gen_stdlib_looks.py): an anchor independent of the product's
compiler for `\\b`, `(?m)^`, `(?m)$`."""
import pytest

import regex_amd as R
from golden_data import stdlib_looks_fixtures
from oracle_py import OracleRegex

FX, TEXT = stdlib_looks_fixtures()


@pytest.mark.parametrize("pat", FX["patterns"])
def test_oracle_find_iter_vs_stdlib(pat):
    o = OracleRegex(R.Regex(pat))
    for (off, n), exp in zip(FX["slices"], FX["find_iter"][pat]):
        assert o.find_iter(TEXT[off:off + n]) == [tuple(x) for x in exp], (pat, off)
