"""MatchType::DfaAnchoredReverse on the CPU (oracle/exec.c): a regex anchored
at the end and not at the start runs the reverse DFA over text[start..] from
the end (exec.rs:671-688, chosen at exec.rs:1175-1177).  The slice hides the
byte before `start`, so a match beginning at `start` whose look-behind the
forward DFA would reject is found (the reference's behaviour, reproduced)."""
import pytest

import regex_amd as R
from oracle_py import OracleRegex


@pytest.mark.parametrize("pat,text,start,exp", [
    (r"(?-u)\bx$", b"ax", 1, (1, 2)),     # forward look-behind: no boundary at 1
    (r"(?m)^x\z", b"ax", 1, (1, 2)),      # forward: no line start at 1
    (r"(?-u)\bx$", b"ax", 0, None),
    (r"(?-u)\bx$", b"a x", 0, (2, 3)),
    (r"\d$", b"abc1", 0, (3, 4)),
    (r"\d$", b"abc1x", 0, None),
    (r"x*$", b"abxx", 1, (2, 4)),
    (r"x*$", b"ab", 0, (2, 2)),
    (r"$", b"abc", 2, (3, 3)),
    (r"(a|ab)$", b"zab", 0, (1, 3)),
])
def test_oracle_anchored_reverse(pat, text, start, exp):
    re = R.Regex(pat)
    info, _ = re.program(2)
    assert info.anchored_end and not info.anchored_start
    o = OracleRegex(re)
    assert o.find(text, start) == exp
    assert o.is_match(text, start) == (exp is not None)
    assert o.shortest_match(text, start) == (None if exp is None else len(text))


def test_not_anchored_reverse_when_anchored_start():
    # ^x$ is anchored at both ends: the forward DFA (no quirk at start > 0)
    o = OracleRegex(R.Regex(r"^x$"))
    assert o.find(b"ax", 1) is None
