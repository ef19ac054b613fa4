"""CPU check of the eager DFA materializer + minimiser: the exported tables,
walked exactly as the HIP kernel walks them, reproduce the reference's golden
answers (find / shortest / is_match / find_iter)."""
import pytest

import regex_amd as R
from dfa_sim import QuitError, find
from golden_data import vectors

V = vectors()


def tables(re):
    f = re.dfa_tables(0)
    r = re.dfa_tables(1)
    return f, r


@pytest.mark.parametrize("v", V["mat"], ids=[x["name"] for x in V["mat"]])
def test_mat_tables(v):
    re = R.Regex(v["re"])
    f, r = tables(re)
    t = bytes.fromhex(v["text"])
    exp = tuple(v["groups"][0]) if v["groups"][0] else None
    try:
        assert find(f, r, t) == exp
        assert find(f, r, t, mode="is_match") == (exp is not None)
        assert (find(f, r, t, mode="shortest") is not None) == (exp is not None)
    except QuitError:
        assert f[0]["quit"] >= 0 and any(b >= 0x80 for b in t)


@pytest.mark.parametrize("v", V["matiter"], ids=[x["name"] for x in V["matiter"]])
def test_matiter_tables(v):
    re = R.Regex(v["re"])
    f, r = tables(re)
    t = bytes.fromhex(v["text"])
    out, last_end, last_match = [], 0, None
    try:
        while last_end <= len(t):
            m = find(f, r, t, last_end)
            if m is None:
                break
            s, e = m
            if s == e:
                last_end = e + 1
                if last_match == e:
                    continue
            else:
                last_end = e
            last_match = e
            out.append((s, e))
    except QuitError:
        return
    assert out == [tuple(m) for m in v["matches"]]


def test_date_dfa_shape():
    info = R.Regex(r"\d{4}-\d{2}-\d{2}").dfa_info(0)
    assert info["ok"] == 1 and info["states"] <= 256 and 11 <= info["hot"] <= 63
