"""CPU check of the find_iter automaton's ASCII shadow (host dfa_build
DfaBuildLimits::ascii_only + prune_unreachable, exported as dfa_tables(5)):
small enough for the all-rows LDS table, and over ASCII text every search
(dfa_sim.find, the kernels' algorithm) answers as the full automaton's; a
search reading a non-ASCII byte quits or answers the same."""
import random
import zlib

import pytest

import regex_amd as R
from dfa_sim import QuitError, find

PATS = [r"\w+", r"(?m)^\w+", r"\pL+\s", r"\w+@\w+\.\w+", r"\w{2,4}", r"[\w.]+@\w+", r"(?m)\w+$"]


def _text(seed, n, nonascii):
    rng = random.Random(seed)
    alpha = [b"a", b"b", b"Z", b"1", b" ", b"\n", b"@", b".", b"_"] + (["é".encode(), b"\xff"] if nonascii else [])
    return b"".join(rng.choices(alpha, k=n))[:n]


@pytest.mark.parametrize("pat", PATS)
def test_ascii_shadow_equals_full_on_ascii(pat):
    re = R.Regex(pat)
    full = re.dfa_tables(2)
    sh = re.dfa_tables(5)
    assert sh is not None, pat
    # the property the shadow exists for: it fits the all-rows LDS table
    # (every state hot, <= 255 of them), the full automaton does not
    i5, i2 = re.dfa_info(5), re.dfa_info(2)
    assert i5["states"] <= 255 and i5["hot"] == i5["states"], (pat, i5)
    assert i2["hot"] < i2["states"], (pat, i2)
    assert i5["quit"] >= 0 and i2["quit"] < 0, pat  # non-ASCII bytes quit the shadow only
    rev = re.dfa_tables(1)
    quits = 0
    for i in range(6):
        t = _text(zlib.crc32(pat.encode()) + i, 120, i % 2 == 1)
        for st in range(len(t) + 1):
            a = find(full, rev, t, st)
            try:
                b = find(sh, rev, t, st)
            except QuitError:
                quits += 1
                continue
            assert a == b, (pat, t, st)
    assert quits > 0, pat


def test_no_shadow_where_not_needed():
    for pat in [r"[a-z]+", r"(?-u)\w+", r"\b\w+\b", r"abc|abd"]:
        assert R.Regex(pat).dfa_info(5) is None, pat
