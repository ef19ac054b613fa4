"""The oracle against a compiler-independent engine: Python's
`re` answers for the BASELINE patterns (the 64 C4 patterns, the C2 date and
C5 email regexes) on ASCII haystacks (tests/golden/gen_stdlib_fixtures.py).
The oracle runs the product compiler's programs, so this pins the parser and
compiler on exactly the patterns the benchmarks time."""
import regex_amd as R
from golden_data import stdlib_fixtures
from oracle_py import OracleRegex

FX = stdlib_fixtures()


def test_c4_set_vs_stdlib():
    c4 = FX["c4"]
    o = OracleRegex(R.RegexSet(c4["patterns"]))
    for line, exp in zip(c4["lines"], c4["matches"]):
        assert o.matches(line.encode()) == exp, line


def test_c4_patterns_one_by_one_vs_stdlib():
    c4 = FX["c4"]
    for j, p in enumerate(c4["patterns"]):
        o = OracleRegex(R.Regex(p))
        for line, exp in zip(c4["lines"][:500], c4["matches"][:500]):
            assert o.is_match(line.encode()) == (j in exp), (p, line)


def test_date_and_email_vs_stdlib():
    for key in ("date", "email"):
        d = FX[key]
        o = OracleRegex(R.Regex(d["pattern"]))
        for h, exp in zip(d["haystacks"], d["find"]):
            assert o.find(h.encode()) == (tuple(exp) if exp else None), (key, h)
    d = FX["email"]
    o = OracleRegex(R.Regex(d["pattern"]))
    for h, exp in zip(d["haystacks"], d["find_iter"]):
        assert o.find_iter(h.encode()) == [tuple(m) for m in exp], h
