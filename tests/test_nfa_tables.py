"""CPU check of the Pike VM closure tables (host/nfa_build.cpp) and of the NFA
kernel's algorithm (tests/nfa_sim.py mirrors nfa_scan.hip): every golden
vector of the reference, including the Unicode word-boundary ones the DFA
quits on, must come out exactly."""
import pytest

import regex_amd as R
from golden_data import vectors
from nfa_sim import NfaSim

V = vectors()


def sim(re):
    return NfaSim(re.nfa_tables(), single=True)


@pytest.mark.parametrize("v", V["mat"], ids=[x["name"] for x in V["mat"]])
def test_mat_nfa(v):
    re = R.Regex(v["re"])
    s = sim(re)
    t = bytes.fromhex(v["text"])
    exp = tuple(v["groups"][0]) if v["groups"][0] else None
    assert s.run(t) == exp
    assert s.run(t, mode="is_match") == (exp is not None)
    assert (s.run(t, mode="shortest") is not None) == (exp is not None)


@pytest.mark.parametrize("v", V["matiter"], ids=[x["name"] for x in V["matiter"]])
def test_matiter_nfa(v):
    s = sim(R.Regex(v["re"]))
    t = bytes.fromhex(v["text"])
    out, last_end, last_match = [], 0, None
    while last_end <= len(t):
        m = s.run(t, last_end)
        if m is None:
            break
        a, e = m
        if a == e:
            last_end = e + 1
            if last_match == e:
                continue
        else:
            last_end = e
        last_match = e
        out.append((a, e))
    assert out == [tuple(m) for m in v["matches"]]


@pytest.mark.parametrize("v", V["matset"] + V["nomatset"],
                         ids=[x["name"] for x in V["matset"] + V["nomatset"]])
def test_set_nfa(v):
    rs = R.RegexSet(v["res"])
    t = bytes.fromhex(v["text"])
    if len(v["res"]) < 2:
        pytest.skip("one-pattern sets run the single-regex engine")
    s = NfaSim(rs.nfa_tables(), single=False)
    mask = s.run(t, mode="set")
    assert sorted(i for i in range(len(v["res"])) if mask >> i & 1) == sorted(v["matches"])


def test_unicode_word_boundary_tables():
    re = R.Regex(r"\bx\b")
    info = re.nfa_tables()[0]
    assert info["unicode_wb"] == 1
    s = sim(re)
    assert s.run("«x".encode()) == (2, 3)
    assert s.run("éxé".encode()) is None
    assert s.run(" x ".encode()) == (1, 2)


# --- seeded differential check against the oracle (DFA -> Quit -> Pike VM) ---
FUZZ_PATTERNS = [r"\b\w+\b", r"\B\w\B", r"(?m)^\w+$", r"a\b|b\B", r"\bfoo\b", r"(?i)\bstra\w+",
                 r"[a-zé]+\b", r"\w+@\w+\.\w+", r"(?-u:\b)x(?-u:\b)", r"(a|ab)(c|bcd)(d*)", r"x*",
                 r"\b", r"(?s).\b.", r"\d+(?:\.\d+)?\b"]
ALPHABET = [b"a", b"b", b"x", b"f", b"o", b"1", b".", b" ", b"\n", b"@", "é".encode(), "ß".encode(),
            "✓".encode(), "𝔸".encode(), b"\xff", b"\xc3", b"_"]


def _texts(seed, n):
    import random
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        k = rng.randint(0, 24)
        out.append(b"".join(rng.choice(ALPHABET) for _ in range(k)))
    return out


@pytest.mark.parametrize("pat", FUZZ_PATTERNS)
def test_nfa_sim_vs_oracle(pat):
    from oracle_py import OracleRegex
    re = R.Regex(pat)
    s = sim(re)
    o = OracleRegex(re)
    import zlib
    for i, t in enumerate(_texts(zlib.crc32(pat.encode()), 150)):
        for start in (0, 1):
            if start > len(t):
                continue
            # the oracle's Pike VM (pikevm.rs restated): the engine the kernel replaces
            exp = o.find_nfa(t, start)
            assert s.run(t, start) == exp, (pat, t, start)
            assert s.run(t, start, mode="is_match") == (exp is not None), (pat, t, start)
            assert s.run(t, start, mode="shortest") == o.shortest_nfa(t, start), (pat, t, start)
