"""CPU check of the captures path: the closure entries' Save lists
(host/nfa_build.cpp, exported by rure_amd_nfa_saves_export) walked the way
the captures kernel walks them (tests/nfa_sim.py CapsSim mirrors
nfa_scan.hip caps_kernel) must give the reference's groups on every golden
`mat!` vector, and agree with the oracle's Pike VM (pikevm.rs restated) and
its read_captures_at dispatch (exec.rs:524-596) on seeded inputs."""
import zlib

import pytest

import regex_amd as R
from golden_data import vectors
from nfa_sim import CapsSim
from oracle_py import OracleRegex

V = vectors()


def caps_sim(re):
    return CapsSim(re.nfa_tables(), re.nfa_saves(), 2 * re.captures_len())


def groups(slots):
    if slots is None:
        return None
    return [None if slots[2 * i] is None or slots[2 * i + 1] is None else (slots[2 * i], slots[2 * i + 1])
            for i in range(len(slots) // 2)]


def bounds(o, t, start, info):
    """The DFA's bounds as caps_kernel receives them (no DFA quit without a
    Unicode word boundary)."""
    return o.find(t, start)


@pytest.mark.parametrize("v", V["mat"], ids=[x["name"] for x in V["mat"]])
def test_mat_captures(v):
    re = R.Regex(v["re"])
    s = caps_sim(re)
    o = OracleRegex(re)
    t = bytes.fromhex(v["text"])
    exp = [tuple(g) if g else None for g in v["groups"]]
    full = groups(s.pike(t, 0))
    assert full == o.captures_nfa(t)
    if not s.info["unicode_wb"]:
        got = groups(s.captures(t, 0, bounds(o, t, 0, s.info)))
        assert got == o.captures(t)
        if got is None:
            assert exp == [None]
        else:
            assert got[:len(exp)] == exp, (v["src"], got, exp)


CAP_PATTERNS = [
    r"(a)(b)?(c)", r"(?P<y>\d{4})-(?P<m>\d{2})-(?P<d>\d{2})", r"(a|ab)(c|bcd)(d*)", r"((a)|b)+",
    r"(a*)+", r"(a*)*b", r"(a+|b+)*c", r"(?:(a)|(b))*", r"(a??)(a*?)", r"(a?)+b", r"(a|b?)+c",
    r"(\w+)@(\w+)\.(\w+)", r"(?m)^(\w+) (\w+)$", r"(a..$)|(a)", r"(ab|a)(bc|c)?$", r"(x)(?-u:\b)",
    r"(?i)(stra)(ss|ß)e", r"([0-9]+)(\.[0-9]+)?", r"(a)|(b)|(c)", r"((((a))))", r"(.)(.)(.)(.)(.)",
    r"^(a+)(b*)", r"(a+)(b*)$",
]
ALPHABET = [b"a", b"b", b"c", b"d", b"x", b"1", b".", b" ", b"\n", b"@", b"s", "ß".encode(), b"\xff"]


def _texts(seed, n):
    import random
    rng = random.Random(seed)
    return [b"".join(rng.choice(ALPHABET) for _ in range(rng.randint(0, 16))) for _ in range(n)]


@pytest.mark.parametrize("pat", CAP_PATTERNS)
def test_caps_sim_vs_oracle(pat):
    re = R.Regex(pat)
    s = caps_sim(re)
    o = OracleRegex(re)
    for t in _texts(zlib.crc32(pat.encode()), 120):
        for start in (0, 2):
            if start > len(t):
                continue
            assert groups(s.pike(t, start)) == o.captures_nfa(t, start), (pat, t, start)
            assert groups(s.captures(t, start, bounds(o, t, start, s.info))) == o.captures(t, start), \
                (pat, t, start)


def test_dispatch_truncation_quirk():
    """exec.rs:861-875 runs the NFA over text[..e'] with e' two characters
    past the DFA's match end; an end-anchored alternative of higher priority
    can then match at e' (the reference returns those groups)."""
    re = R.Regex(r"(a..$)|(a)")
    o = OracleRegex(re)
    assert o.find(b"abcd") == (0, 1)
    assert o.captures(b"abcd") == [(0, 3), (0, 3), None]
    assert o.captures_nfa(b"abcd") == [(0, 1), None, (0, 1)]
    s = caps_sim(re)
    assert groups(s.captures(b"abcd", 0, (0, 1))) == [(0, 3), (0, 3), None]


def test_capture_names():
    re = R.Regex(r"(?P<y>\d{4})-(\d{2})-(?P<d>\d{2})")
    assert re.captures_len() == 4
    assert re.capture_names() == [None, "y", None, "d"]
    assert re.capture_name_index("y") == 1 and re.capture_name_index("d") == 3
    assert re.capture_name_index("m") is None
