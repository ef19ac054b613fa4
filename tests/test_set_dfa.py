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
