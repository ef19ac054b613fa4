"""Host side of replace: `$` reference parsing and expansion (expand.rs)
against the reference's own find_cap_ref cases (expand.rs:195-207), and the
CPU restatement of split/splitn/replacen (tests/replace_ref.py) against the
reference's replace! / split! vectors through the oracle."""
import pytest

import regex_amd as R
from golden_data import vectors
from oracle_py import OracleRegex
import replace_ref as RR

V = vectors()


@pytest.mark.parametrize("text,exp", [
    ("$foo", ("foo", 4)), ("${foo}", ("foo", 6)), ("$0", (0, 2)), ("$5", (5, 2)), ("$10", (10, 3)),
    ("$42a", ("42a", 4)), ("${42}a", (42, 5)), ("${42", None), ("${42 ", None), (" $0 ", None), ("$", None),
    (" ", None), ("", None)])
def test_find_cap_ref(text, exp):
    assert R._find_cap_ref(text.encode()) == exp


def test_expand_by_hand():
    text = b"abc 123"
    g = [(0, 7), (0, 3), (4, 7)]
    names = [None, "a", "b"]
    assert R.expand(g, names, b"$b$a", text) == b"123abc"
    assert R.expand(g, names, b"z$bz$az", text) == b"z"
    assert R.expand(g, names, b".$b.$a.", text) == b".123.abc."
    assert R.expand(g, names, b"$$1 $$foo ${1}x $", text) == b"$1 $foo abcx $"
    assert R.expand([(0, 1), None], [None, None], b"[$1]", b"a") == b"[]"


@pytest.mark.parametrize("v", V["replace"], ids=[x["name"] for x in V["replace"]])
def test_replace_vectors_oracle(v):
    re = R.Regex(v["re"])
    o = OracleRegex(re)
    text, rep = bytes.fromhex(v["text"]), bytes.fromhex(v["rep"])
    limit = 1 if v["which"] == "replace" else 0
    got = RR.replacen(o, re.capture_names(), text, limit, rep, v["mode"] == "literal")
    assert got == bytes.fromhex(v["result"]), v["src"]


@pytest.mark.parametrize("v", V["split"], ids=[x["name"] for x in V["split"]])
def test_split_vectors_oracle(v):
    o = OracleRegex(R.Regex(v["re"]))
    assert RR.split(o, bytes.fromhex(v["text"])) == [bytes.fromhex(f) for f in v["fields"]], v["src"]


def test_splitn_rules_oracle():
    """re_bytes.rs:729-749 walked by hand: the remainder field may be empty."""
    o = OracleRegex(R.Regex(r","))
    assert RR.splitn(o, b"a,b", 0) == []
    assert RR.splitn(o, b"a,b", 1) == [b"a,b"]
    assert RR.splitn(o, b"a,b", 2) == [b"a", b"b"]
    assert RR.splitn(o, b"a,b", 3) == [b"a", b"b", b""]
    assert RR.splitn(o, b"a,b", 4) == [b"a", b"b"]
    assert RR.splitn(o, b"a,", 3) == [b"a"]
    assert RR.splitn(o, b"a,", 2) == [b"a", b""]
    o = OracleRegex(R.Regex(r"\W+"))
    assert RR.splitn(o, b"Hey! How are you?", 3) == [b"Hey", b"How", b"are you?"]
