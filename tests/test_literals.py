"""CPU checks of the literal find_iter engine (host/literals.cpp +
iter_spec_lit_kernel): the finite string set read off the NFA program, in
priority order, iterated greedily (first literal in order that matches at the
leftmost start, next search at its end — re_trait.rs:197-221) must give the
oracle's find_iter exactly.  TEST INFRASTRUCTURE (oracle = the checker)."""
import random
import zlib

import pytest

import regex_amd as R
from golden_data import corpus, known_counts
from oracle_py import OracleRegex

LITERAL = [r"agggtaaa|tttaccct", r"[cgt]gggtaaa|tttaccc[acg]", r"agggtaa[cgt]|[acg]ttaccct", r"a|ab", r"ab|a",
           r"aa", r"a", r"(?i)holm", r"Sherlock|Holmes|Watson", r"foo(bar)?", r"(foo)??bar", r"x(a|ab)(c|bcd)",
           r"[0-3]{2}", r"abc|abd|ab", r"é", r"(?i)k"]
NOT_LITERAL = [r"[0-9]{2}", r"\w+", r"a+", r"x*", r"", r"^abc", r"abc$", r"\bfoo", r"a?", r"[a-z]{3}x{0,2}y"]


def greedy(lits, text):
    out, p = [], 0
    while p < len(text):
        hit = None
        for i in range(p, len(text)):
            for lit in lits:
                if text.startswith(lit, i):
                    hit = (i, i + len(lit))
                    break
            if hit:
                break
        if not hit:
            break
        out.append(hit)
        p = hit[1]
    return out


def texts(pat):
    rng = random.Random(zlib.crc32(pat.encode()))
    alpha = [b"a", b"b", b"c", b"d", b"x", b"g", b"t", b"foo", b"bar", b"1", b"2", b"k", b"K",
             "é".encode(), b"\xe2\x84\xaa", b"Holmes", b"holmes", b" "]
    yield corpus("sherlock")[:20000]
    yield corpus("regexdna")[:20000]
    for _ in range(4):
        yield b"".join(rng.choice(alpha) for _ in range(400))


@pytest.mark.parametrize("pat", LITERAL)
def test_literal_engine_matches_oracle(pat):
    re = R.Regex(pat)
    lits = re.literals()
    assert lits, pat
    o = OracleRegex(re)
    for t in texts(pat):
        assert greedy(lits, t) == o.find_iter(t), pat


@pytest.mark.parametrize("pat", NOT_LITERAL)
def test_not_a_string_set(pat):
    assert R.Regex(pat).literals() is None


def test_priority_order():
    assert R.Regex(r"a|ab").literals() == [b"a", b"ab"]
    assert R.Regex(r"ab|a").literals() == [b"ab", b"a"]
    assert R.Regex(r"foo(bar)?").literals() == [b"foobar", b"foo"]
    assert R.Regex(r"foo(bar)??").literals() == [b"foo", b"foobar"]
    assert len(R.Regex(r"(?i)holm").literals()) == 16
    assert R.Regex(r"(?i)holmes").literals() is None  # 96 strings (s folds to U+017F too)


def test_regexdna_variants_are_string_sets():
    for v in known_counts()["regexdna"]["variants"]:
        lits = R.Regex(v["re"]).literals()
        assert lits and all(len(x) == 8 for x in lits), v["re"]


def test_long_literals_second_filter():
    """Literals of >= 8 bytes get the bytes-4..7 bitmap (C3 variants)."""
    lits = R.Regex(r"agggtaa[cgt]|[acg]ttaccct").literals()
    assert min(len(x) for x in lits) >= 8


def test_suffix_walk_quirk_in_oracle():
    """MatchType::DfaSuffix (exec.rs:725-794) restated in the oracle: the
    walk over the longest common suffix's occurrences decides at the first
    "ing" of `xaaingbing` (`a+ing`, start 1), where a leftmost-first search
    finds the longer `xa*ingb*ing` from 0."""
    re = R.Regex(r"xa*ingb*ing|a+ing")
    assert re.match_info()["match_type"] == "DfaSuffix"
    o = OracleRegex(re)
    assert o.find(b"xaaingbing") == (1, 6)
    assert o.find_iter(b"xaaingbing xaing") == [(1, 6), (12, 16)]
