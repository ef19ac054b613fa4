"""Host side of the big (u32 column form) automata: regexes whose DFA
exceeds the u16 tables get both directions built with the larger budget
(dfa_build.cpp kBigDfaRawStates), and the column form steps exactly like
the 256-wide form of the same program (checked on a DFA both can hold)."""
import pytest

import regex_amd as R

BIG = [r"[a-q][^u-z]{13}x", r"(?:a|b)*a(?:a|b){14}", r"(?i)[a-q][^u-z]{13}x"]


@pytest.mark.parametrize("pat", BIG)
def test_big_automaton_built(pat):
    re = R.Regex(pat)
    assert re.dfa_info(0) is None  # past the u16 tables
    f, r = re.dfa_info(3), re.dfa_info(4)
    assert f is not None and f["states"] > 65535, f
    assert r is not None and r["quit"] == -1


@pytest.mark.parametrize("pat", [r"\w+@\w+", r"[a-q][^u-z]{3}x", r"(?i)holmes"])
def test_small_automaton_has_no_big_form(pat):
    re = R.Regex(pat)
    assert re.dfa_info(0) is not None
    assert re.dfa_info(3) is None


def test_unicode_word_boundary_keeps_pike():
    # quit states (non-ASCII bytes under a Unicode \b): no big automaton
    re = R.Regex(r"[a-q][^u-z]{13}x\b")
    assert re.dfa_info(0) is None
    assert re.dfa_info(3) is None
