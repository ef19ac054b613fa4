"""GPU parity of the wavefront Pike VM kernel (nfa_scan.hip): the DFA-quit
fallback (Unicode word boundaries on non-ASCII input), the NFA-only path
(automata too large to materialise) and sets, against the oracle's
full engine dispatch (exec.rs: DFA -> Quit -> Pike VM), bit-exact."""
import random
import zlib

import numpy as np
import pytest

import regex_amd as R
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

ALPHABET = [b"a", b"b", b"x", b"f", b"o", b"1", b"2", b".", b" ", b"\n", b"@", b"-", "é".encode(),
            "ß".encode(), "✓".encode(), "𝔸".encode(), b"\xff", b"\xc3", b"_"]

QUIT_PATTERNS = [r"\b\w+\b", r"\B\w\B", r"\bfoo\b", r"(?i)\bab\w*", r"[a-zé]+\b", r"\b\d+\b",
                 r"(?m)^\w+\b$", r"\b", r"x\b|\bo"]
BIG_PATTERNS = [r"(?-u:[ab])*a(?-u:[ab]){17}", r"(?-u:[ab])*b(?-u:[ab]){16}x"]


def ragged(seed, n, maxlen):
    rng = random.Random(seed)
    hs = [b"".join(rng.choice(ALPHABET) for _ in range(rng.randint(0, maxlen))) for _ in range(n)]
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(h) for h in hs])
    return hs, np.frombuffer(b"".join(hs) + b"\0" * 16, dtype=np.uint8).copy(), offs


def check_regex_batch(re, hs, buf, offs, cuda, start=0):
    import torch
    o = OracleRegex(re)
    dev = torch.from_numpy(buf).to(cuda)
    doff = torch.from_numpy(offs).to(cuda)
    got = re.find_batch(dev, offsets=doff, start=start).cpu().numpy().astype(np.uint64)
    ism = re.is_match_batch(dev, offsets=doff, start=start).cpu().numpy()
    sho = re.shortest_match_batch(dev, offsets=doff, start=start).cpu().numpy().astype(np.uint64)
    for i, t in enumerate(hs):
        exp = o.find(t, start) if start <= len(t) else None
        g = None if int(got[i, 0]) == R.NONE else (int(got[i, 0]), int(got[i, 1]))
        assert g == exp, (re.pattern, t, start, g, exp)
        assert bool(ism[i]) == (o.is_match(t, start) if start <= len(t) else False), (re.pattern, t)
        es = o.shortest_match(t, start) if start <= len(t) else None
        gs = None if int(sho[i]) == R.NONE else int(sho[i])
        assert gs == es, (re.pattern, t, start, gs, es)


@pytest.mark.parametrize("pat", QUIT_PATTERNS)
@pytest.mark.parametrize("start", [0, 1])
def test_quit_fallback_batch(cuda, pat, start):
    re = R.Regex(pat)
    assert re.uses_dfa() and re.dfa_info(0)["quit"] >= 0
    hs, buf, offs = ragged(zlib.crc32(pat.encode()) + start, 600, 40)
    check_regex_batch(re, hs, buf, offs, cuda, start)


@pytest.mark.parametrize("pat", BIG_PATTERNS)
def test_nfa_only_batch(cuda, pat):
    re = R.Regex(pat)
    assert not re.uses_dfa()
    rng = random.Random(7)
    hs = [bytes(rng.choice(b"ab") for _ in range(rng.randint(0, 60))) + rng.choice([b"", b"x"])
          for _ in range(300)]
    offs = np.zeros(len(hs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(h) for h in hs])
    buf = np.frombuffer(b"".join(hs) + b"\0" * 16, dtype=np.uint8).copy()
    check_regex_batch(re, hs, buf, offs, cuda)


def test_nfa_single_calls(cuda):
    re = R.Regex(r"\b\w+\b")
    o = OracleRegex(re)
    for t in ["héllo wörld", "«x»", "ab✓cd", "𝔸𝔸 b"]:
        tb = t.encode()
        assert re.find(tb) == o.find(tb)
        assert re.find_iter(tb) == o.find_iter(tb)
        assert re.is_match(tb) == o.is_match(tb)


@pytest.mark.parametrize("pats", [[r"\bfoo\b", r"\w+", r"ß"], [r"\bx", r"o\b", r"\d\b", r"é"]])
def test_set_quit_fallback_batch(cuda, pats):
    import torch
    rs = R.RegexSet(pats)
    o = OracleRegex(rs)
    hs, buf, offs = ragged(zlib.crc32("|".join(pats).encode()), 500, 30)
    got = rs.matches_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy()
    for i, t in enumerate(hs):
        exp = o.matches(t)
        g = [j for j in range(len(pats)) if (int(got[i]) >> j) & 1]
        assert g == exp, (pats, t, g, exp)


def test_set_nfa_only_batch(cuda):
    import torch
    pats = [r"(?-u:[ab])*a(?-u:[ab]){17}", r"bb", r"^a"]
    rs = R.RegexSet(pats)
    assert not rs.uses_dfa()
    o = OracleRegex(rs)
    rng = random.Random(3)
    hs = [bytes(rng.choice(b"ab") for _ in range(rng.randint(0, 50))) for _ in range(200)]
    offs = np.zeros(len(hs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(h) for h in hs])
    buf = np.frombuffer(b"".join(hs) + b"\0" * 16, dtype=np.uint8).copy()
    got = rs.matches_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy()
    for i, t in enumerate(hs):
        exp = o.matches(t)
        assert [j for j in range(3) if (int(got[i]) >> j) & 1] == exp, t
