"""The reference's golden vectors through the product's GPU path (C ABI ->
HIP kernels): rure_find / rure_is_match / rure_shortest_match / rure_iter_next
/ rure_set_matches semantics, bit-exact."""
import pytest

import regex_amd as R
from golden_data import known_counts, vectors, corpus

pytestmark = pytest.mark.gpu
V = vectors()


@pytest.mark.parametrize("v", V["mat"], ids=[x["name"] for x in V["mat"]])
def test_mat_gpu(cuda, v):
    re = R.Regex(v["re"])
    t = bytes.fromhex(v["text"])
    exp = tuple(v["groups"][0]) if v["groups"][0] else None
    assert re.find(t) == exp
    assert re.is_match(t) == (exp is not None)
    assert (re.shortest_match(t) is not None) == (exp is not None)


@pytest.mark.parametrize("v", V["matiter"], ids=[x["name"] for x in V["matiter"]])
def test_matiter_gpu(cuda, v):
    re = R.Regex(v["re"])
    t = bytes.fromhex(v["text"])
    assert re.find_iter(t) == [tuple(m) for m in v["matches"]]


@pytest.mark.parametrize("v", V["matset"] + V["nomatset"], ids=[x["name"] for x in V["matset"] + V["nomatset"]])
def test_matset_gpu(cuda, v):
    s = R.RegexSet(v["res"])
    t = bytes.fromhex(v["text"])
    assert s.matches(t) == v["matches"]
    assert s.is_match(t) == bool(v["matches"])


@pytest.mark.parametrize("v", V["ismatch"], ids=[x["name"] for x in V["ismatch"]])
def test_ismatch_gpu(cuda, v):
    assert R.Regex(v["re"]).is_match(bytes.fromhex(v["text"])) == v["expect"]
