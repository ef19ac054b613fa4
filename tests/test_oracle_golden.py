"""Pins the CPU oracle (and the host compiler feeding it) against the
reference's own golden vectors: every mat!/matiter!/matset!/nomatset!/
ismatch!/noparse! of the bytes::Regex test target, the sherlock find_iter
counts and the regex-dna shootout known answer.  CPU only."""
import pytest

import regex_amd as R
from golden_data import corpus, known_counts, vectors
from oracle_py import OracleRegex

V = vectors()


def _ids(xs):
    return [x["name"] for x in xs]


@pytest.mark.parametrize("v", V["mat"], ids=_ids(V["mat"]))
def test_mat(v):
    text = bytes.fromhex(v["text"])
    re = R.Regex(v["re"])
    o = OracleRegex(re)
    exp = [tuple(g) if g else None for g in v["groups"]]
    got_find = o.find(text)
    assert got_find == exp[0], (v["src"], got_find, exp)
    assert o.find_nfa(text) == exp[0]
    assert o.is_match(text) == (exp[0] is not None)
    assert (o.shortest_match(text) is not None) == (exp[0] is not None)
    for caps in (o.captures(text), o.captures_nfa(text)):
        if caps is None:
            assert exp == [None]
        else:
            assert caps[:len(exp)] == exp, (v["src"], caps, exp)


@pytest.mark.parametrize("v", V["matiter"], ids=_ids(V["matiter"]))
def test_matiter(v):
    text = bytes.fromhex(v["text"])
    o = OracleRegex(R.Regex(v["re"]))
    assert o.find_iter(text) == [tuple(m) for m in v["matches"]], v["src"]


@pytest.mark.parametrize("v", V["matset"] + V["nomatset"], ids=_ids(V["matset"] + V["nomatset"]))
def test_matset(v):
    text = bytes.fromhex(v["text"])
    s = R.RegexSet(v["res"])
    if len(v["res"]) == 0:
        return
    o = OracleRegex(s) if len(v["res"]) > 1 else None
    if o is None:
        r1 = OracleRegex(R.Regex(v["res"][0]))
        got = [0] if r1.is_match(text) else []
    else:
        got = o.matches(text)
        assert o.matches(text, nfa=True) == got
    assert got == v["matches"], v["src"]


@pytest.mark.parametrize("v", V["ismatch"], ids=_ids(V["ismatch"]))
def test_ismatch(v):
    o = OracleRegex(R.Regex(v["re"]))
    assert o.is_match(bytes.fromhex(v["text"])) == v["expect"]


@pytest.mark.parametrize("v", V["noparse"], ids=_ids(V["noparse"]))
def test_noparse(v):
    with pytest.raises(R.Error):
        R.Regex(v["re"])


KC = known_counts()


@pytest.mark.parametrize("v", KC["sherlock"], ids=[x["name"] for x in KC["sherlock"]])
def test_sherlock_counts(v):
    text = corpus("sherlock")
    o = OracleRegex(R.Regex(v["re"]))
    assert len(o.find_iter(text)) == v["count"], v["src"]


def replace_all(o, text, rep=b""):
    out, last = [], 0
    for s, e in o.find_iter(text):
        out.append(text[last:s])
        out.append(rep)
        last = e
    out.append(text[last:])
    return b"".join(out)


def test_regexdna_known_answer():
    dna = KC["regexdna"]
    text = corpus("regexdna")
    assert len(text) == dna["input_len"]
    seq = replace_all(OracleRegex(R.Regex(dna["strip"])), text)
    assert len(seq) == dna["stripped_len"]
    for v in dna["variants"]:
        assert len(OracleRegex(R.Regex(v["re"])).find_iter(seq)) == v["count"], v["re"]
    subst = [("B", b"(c|g|t)"), ("D", b"(a|g|t)"), ("H", b"(a|c|t)"), ("K", b"(g|t)"), ("M", b"(a|c)"),
             ("N", b"(a|c|g|t)"), ("R", b"(a|g)"), ("S", b"(c|g)"), ("V", b"(a|c|g)"), ("W", b"(a|t)"),
             ("Y", b"(c|t)")]
    for pat, rep in subst:
        seq = replace_all(OracleRegex(R.Regex(pat)), seq, rep)
    assert len(seq) == dna["substituted_len"]
