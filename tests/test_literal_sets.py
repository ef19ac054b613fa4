"""The reference's literal extraction (regex-syntax/src/literals.rs) restated
in host/literal_sets.cpp, pinned by regex-syntax's own test vectors
(tests/golden/literal_vectors.json, extracted by extract_literal_vectors.py):
prefixes / suffixes with default and exhausted limits (both the Unicode and
the bytes parse, as the reference's test_lit! runs them), unambiguous
prefixes, longest common prefix / suffix.  Then the engine choice built on
them (exec.rs:1130-1210) on hand-checked cases."""
import json
import os

import pytest

import regex_amd as R

HERE = os.path.dirname(os.path.abspath(__file__))
V = json.load(open(os.path.join(HERE, "golden", "literal_vectors.json")))


def esc(b):
    """Rust's ascii::escape_default per byte (the tests' escape_bytes)."""
    out = []
    for x in b:
        c = chr(x)
        if c == "\t":
            out.append("\\t")
        elif c == "\r":
            out.append("\\r")
        elif c == "\n":
            out.append("\\n")
        elif c == "\\":
            out.append("\\\\")
        elif c == "'":
            out.append("\\'")
        elif c == '"':
            out.append('\\"')
        elif 0x20 <= x < 0x7F:
            out.append(c)
        else:
            out.append("\\x%02x" % x)
    return "".join(out)


def as_expected(lits):
    return [["C" if cut else "M", esc(v)] for v, cut in lits]


@pytest.mark.parametrize("case", V["lit"], ids=[c["name"] for c in V["lit"]])
def test_lit(case):
    for unicode in (True, False):
        got = R.syntax_literals(case["re"], case["which"], unicode=unicode)
        assert as_expected(got) == case["expected"], (case["re"], unicode)


@pytest.mark.parametrize("case", V["exhausted"], ids=[c["name"] for c in V["exhausted"]])
def test_exhausted(case):
    for unicode in (True, False):
        got = R.syntax_literals(case["re"], case["which"], unicode=unicode, limit_size=20, limit_class=10)
        assert as_expected(got) == case["expected"], (case["re"], unicode)


def unesc(s):
    return s.encode("latin-1").decode("unicode_escape").encode("latin-1")


@pytest.mark.parametrize("case", V["unamb"], ids=[c["name"] for c in V["unamb"]])
def test_unambiguous(case):
    given = [(unesc(v), k == "C") for k, v in case["given"]]
    got = R.literals_op("unambiguous_prefixes", given)
    assert as_expected(got) == case["expected"]


@pytest.mark.parametrize("kind", ["lcp", "lcs"])
def test_lcp_lcs(kind):
    for case in V[kind]:
        given = [(g.encode("latin-1"), False) for g in case["given"]]
        assert esc(R.literals_op(kind, given)) == case["expected"], case["name"]


# exec.rs:1130-1210 on hand-checked regexes (the literal sets they rest on:
# exec.rs:209-271 with the sets' unambiguous forms)
MATCH_TYPES = [
    (r"abc", "Literal(Unanchored)"),
    (r"Sherlock|Holmes|Watson", "Literal(Unanchored)"),
    (r"^abc", "Literal(AnchoredStart)"),
    (r"^(?:abc|xyz)", "Literal(AnchoredStart)"),
    (r"(?:abc|xyz)$", "Literal(AnchoredEnd)"),
    (r"\d{4}-\d{2}-\d{2}", "Dfa"),
    (r"\w+@\w+\.\w+", "Dfa"),
    (r"\w+\s+Holmes", "DfaSuffix"),
    (r"[a-z]+ing", "DfaSuffix"),
    (r"a!Xbcd.Xbcd|(?-u:\b)Xbcd", "DfaSuffix"),
    (r"Holmes\w+", "Dfa"),                  # lcp "Holmes" wins over no suffix
    (r"[a-z]+ing$", "DfaAnchoredReverse"),
    (r"a|ab", "Dfa"),                       # "a" is a prefix of "ab": cut, not complete
    (r"(?:a|b|c|d|e|f|g|h|i|j|k|l|m|n|o|p|q|r|s|t|u|v|w|x|y|z)x", "Literal(Unanchored)"),
    (r">[^\n]*\n|\n", "Dfa"),
    (r"agggtaaa|tttaccct", "Literal(Unanchored)"),
]


@pytest.mark.parametrize("pat,mt", MATCH_TYPES)
def test_match_type(pat, mt):
    assert R.Regex(pat).match_info()["match_type"] == mt


def test_empty_prefix_matcher_quirk_inputs():
    # 26 first bytes: the prefix searcher is Matcher::Empty (literals.rs:201-209)
    # while the suffix set is complete -> Literal(Unanchored) searched with the
    # empty prefix matcher (exec.rs:1156-1165, literals.rs:92-96)
    i = R.Regex(r"(?:a|b|c|d|e|f|g|h|i|j|k|l|m|n|o|p|q|r|s|t|u|v|w|x|y|z)x").match_info()
    assert i["prefix_matcher"] == 0 and i["prefix_len"] == 0 and not i["prefix_complete"]
    assert i["suffix_complete"] and i["suffix_matcher"] == 3 and i["suffix_len"] == 26
