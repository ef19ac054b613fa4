"""CPU check of the set DFA (per-step match masks, host/dfa_build.cpp) walked
as the set kernel walks it, against the reference's set vectors and the
oracle's forward_many (carried-match lazy DFA) on seeded texts."""
import random
import zlib

import pytest

import regex_amd as R
from dfa_sim import QuitError, set_matches
from golden_data import vectors
from oracle_py import OracleRegex

V = vectors()
SETS = V["matset"] + V["nomatset"]


def tables(rs):
    t = rs.dfa_tables()
    t[0]["n"] = len(rs)
    return t


@pytest.mark.parametrize("v", SETS, ids=[x["name"] for x in SETS])
def test_set_vectors(v):
    if len(v["res"]) < 2:
        pytest.skip("one-pattern sets run the single-regex engine")
    rs = R.RegexSet(v["res"])
    t = bytes.fromhex(v["text"])
    try:
        m = set_matches(tables(rs), t)
    except QuitError:
        assert rs.dfa_info()["quit"] >= 0
        return
    assert [i for i in range(len(v["res"])) if m >> i & 1] == sorted(v["matches"])


FUZZ_SETS = [[r"a", r"b", r"ab"], [r"^a", r"a$", r"(?m)^b$", r"x*"], [r"\d+", r"[a-c]{2}", r"c\.d", r"^$"],
             [r"(?-u:\b)ab", r"ba(?-u:\B)", r"a+b+", r"z"], [r"(?i)AB", r"cd|de", r"e(?s:.)f", r"\n"]]


@pytest.mark.parametrize("pats", FUZZ_SETS)
def test_set_dfa_vs_oracle(pats):
    rs = R.RegexSet(pats)
    tb = tables(rs)
    o = OracleRegex(rs)
    rng = random.Random(zlib.crc32("|".join(pats).encode()))
    for _ in range(300):
        t = bytes(rng.choice(b"abcdefz.1\n AB") for _ in range(rng.randint(0, 20)))
        for start in (0, 1):
            m = set_matches(tb, t, start)
            exp = o.matches(t, start) if start <= len(t) else []
            assert [i for i in range(len(pats)) if m >> i & 1] == exp, (pats, t, start)


def test_core_form_c4_lines():
    """The 64-pattern C4 set in core form, walked as set_core_kernel walks it,
    against the oracle on seeded log lines."""
    import numpy as np
    from dfa_sim import core_set_matches
    from regex_amd.workloads import C4_PATTERNS, log_lines_host
    rs = R.RegexSet(C4_PATTERNS)
    ct = rs.core_tables()
    T, hot = ct[2], ct[0]["hot"]
    assert all(int(T[r, -1]) == r << 6 for r in range(hot))  # identity column
    assert ct is not None and ct[0]["hot"] > 500
    buf, offs = log_lines_host(400, seed=77)
    o = OracleRegex(rs)
    for i in range(400):
        t = bytes(buf[offs[i]:offs[i + 1]])
        m = core_set_matches(ct, t, n=len(C4_PATTERNS))
        assert [j for j in range(64) if m >> j & 1] == o.matches(t), i


def test_core_form_fuzz():
    """A set large enough for the core form, on texts with line anchors,
    word boundaries (ASCII) and overlapping matches."""
    from dfa_sim import core_set_matches
    pats = [r"[a-c]+\d", r"\d{2,3}", r"(?m)^ab", r"(?m)c$", r"(?-u:\b)b", r"a.c", r"bb|cc", r"[0-9a-f]{4}",
            r"x\d*y", r"(?i)ABC", r"c\nb", r"a+b+c+"]
    rs = R.RegexSet(pats)
    ct = rs.core_tables()
    if ct is None:
        pytest.skip("set small enough for the byte-row kernel")
    o = OracleRegex(rs)
    rng = random.Random(1234)
    for _ in range(400):
        t = bytes(rng.choice(b"abcdefxy0123\n ABC") for _ in range(rng.randint(0, 60)))
        m = core_set_matches(ct, t, n=len(pats))
        assert [j for j in range(len(pats)) if m >> j & 1] == o.matches(t), t
