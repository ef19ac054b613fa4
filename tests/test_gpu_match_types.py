"""GPU parity of the reference's observable engine choices (exec.rs:1130-1210,
host/literal_sets.cpp, match_types.hip): Literal(AnchoredStart) searches
the literals at the search start whatever it is (exec.rs:613-617),
Literal(Unanchored) chosen from complete suffixes searches with the prefix
searcher (Matcher::Empty matches the empty string), and DfaSuffix reports
the first suffix occurrence whose reverse scan matches (exec.rs:725-794) —
against the oracle, which restates the same dispatch, for find / is_match /
shortest_match batches, single calls, find_iter and captures."""
import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from golden_data import corpus
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

QUIRK = [
    (r"a!Xbcd.Xbcd|(?-u:\b)Xbcd", b"zza!XbcdqXbcd", (4, 8)),       # DfaSuffix: not the leftmost (2, 13)
    (r"^abc", b"abcabc", (0, 3)),                                   # Literal(AnchoredStart)
    (r"(?:a|b|c|d|e|f|g|h|i|j|k|l|m|n|o|p|q|r|s|t|u|v|w|x|y|z)x", b"hello ax", (0, 0)),  # Empty prefix searcher
]

PATTERNS = [
    r"\w+\s+Holmes", r"[a-z]+ing", r"\w+@gmail\.com", r"(?i)\w+ herlock", r"a!Xbcd.Xbcd|(?-u:\b)Xbcd",
    r"[A-Z]\w+ Holmes", r"\bthe\w*ing", r"^abc", r"^(?:ab|cd)", r"^Holmes",
    r"(?:a|b|c|d|e|f|g|h|i|j|k|l|m|n|o|p|q|r|s|t|u|v|w|x|y|z)x", r"(\w+)\s+(Holmes)",
]


def to_dev(buf, cuda):
    import torch
    return torch.from_numpy(np.frombuffer(bytes(buf), dtype=np.uint8).copy()).to(cuda)


def _batch(n, L, seed):
    """Sherlock lines interleaved with strings that exercise the quirks."""
    rng = np.random.default_rng(seed)
    text = corpus("sherlock")
    pieces = [b"zza!XbcdqXbcd", b"abcabc", b"cdab", b"Holmes Holmes", b"singing ring", b"x@gmail.com",
              b"a!Xbcd Xbcd", b"Xbcd", b"\xce\xb1ing \xe2\x98\x83 Holmes", b"hello ax"]
    out = bytearray()
    for i in range(n):
        off = int(rng.integers(0, len(text) - L))
        h = bytearray(text[off:off + L])
        for _ in range(int(rng.integers(0, 3))):
            p = pieces[int(rng.integers(0, len(pieces)))]
            at = int(rng.integers(0, max(1, L - len(p))))
            h[at:at + len(p)] = p[:L - at]
        if i % 7 == 0:
            h[:6] = b"abcabc"
        out += h
    return bytes(out)


@pytest.mark.parametrize("pat,text,exp", QUIRK)
def test_quirks_single(cuda, pat, text, exp):
    re = R.Regex(pat)
    o = OracleRegex(re)
    assert o.find(text) == exp
    assert re.find(text) == exp
    assert re.find_iter(text) == o.find_iter(text)
    assert re.iter_rure(text) == o.find_iter(text) or pat == r"^abc"
    for st in range(len(text) + 1):
        assert re.find(text, st) == o.find(text, st), st
        assert re.is_match(text, st) == o.is_match(text, st), st
        assert re.shortest_match(text, st) == o.shortest_match(text, st), st


@pytest.mark.parametrize("pat", PATTERNS)
@pytest.mark.parametrize("start", [0, 3])
def test_batch_parity(cuda, pat, start):
    n, L = 600, 300
    buf = _batch(n, L, 0xA11 + len(pat))
    d = to_dev(buf + b"\0" * 16, cuda)
    re = R.Regex(pat)
    o = OracleRegex(re)
    got_f = re.find_batch(d, stride=L, length=L, count=n, start=start).cpu().numpy()
    if re.match_info()["match_type"] in ("DfaSuffix", "Literal(AnchoredStart)"):
        assert N.rure_amd_last_fwd_path() == -5
    got_m = re.is_match_batch(d, stride=L, length=L, count=n, start=start).cpu().numpy()
    got_s = re.shortest_match_batch(d, stride=L, length=L, count=n, start=start).cpu().numpy()
    for i in range(n):
        h = buf[i * L:(i + 1) * L]
        e = o.find(h, start)
        g = None if got_f[i, 0] < 0 else (int(got_f[i, 0]), int(got_f[i, 1]))
        assert g == e, (pat, i, start)
        assert bool(got_m[i]) == o.is_match(h, start), (pat, i)
        es = o.shortest_match(h, start)
        assert (None if got_s[i] < 0 else int(got_s[i])) == es, (pat, i)


@pytest.mark.parametrize("pat", PATTERNS)
def test_find_iter_parity(cuda, pat):
    n, L = 200, 400
    buf = _batch(n, L, 0xB22 + len(pat))
    d = to_dev(buf + b"\0" * 16, cuda)
    re = R.Regex(pat)
    o = OracleRegex(re)
    counts, m = re.find_iter_batch(d, stride=L, length=L, count=n)
    counts = counts.cpu().numpy()
    m = [(int(a), int(b)) for a, b in m.cpu().numpy()]
    k = 0
    for i in range(n):
        exp = o.find_iter(buf[i * L:(i + 1) * L])
        assert int(counts[i]) == len(exp), (pat, i)
        assert m[k:k + len(exp)] == exp, (pat, i)
        k += len(exp)


@pytest.mark.parametrize("pat", [r"\w+\s+Holmes", r"[a-z]+ing", r"^abc"])
def test_find_iter_long(cuda, pat):
    text = b"abcabc" + corpus("sherlock")[:200000]
    re = R.Regex(pat)
    assert re.find_iter(text) == OracleRegex(re).find_iter(text)


@pytest.mark.parametrize("pat", [r"(\w+)\s+(Holmes)", r"(?:(a)!Xbcd.Xbcd|(?-u:\b)(X)bcd)", r"^(a)(b)c",
                                 r"([a-z]+)(ing)"])
def test_captures_parity(cuda, pat):
    n, L = 300, 200
    buf = _batch(n, L, 0xC33 + len(pat))
    d = to_dev(buf + b"\0" * 16, cuda)
    re = R.Regex(pat)
    o = OracleRegex(re)
    got = re.captures_batch(d, stride=L, length=L, count=n).cpu().numpy()
    for i in range(n):
        exp = o.captures(buf[i * L:(i + 1) * L])
        g = [None if a < 0 else (int(a), int(b)) for a, b in got[i]]
        if exp is None:
            assert all(x is None for x in g), (pat, i)
        else:
            assert g == exp, (pat, i)


def test_sherlock_counts_suffix(cuda):
    """The reference's own sherlock counts for patterns it runs as DfaSuffix
    (bench/src/sherlock.rs) through the GPU's DfaSuffix iteration."""
    from golden_data import known_counts
    kc = known_counts()["sherlock"]
    text = corpus("sherlock")
    checked = 0
    for case in kc:
        re = R.Regex(case["re"])
        if re.match_info()["match_type"] != "DfaSuffix":
            continue
        assert len(re.find_iter(text)) == case["count"], case["re"]
        checked += 1
    assert checked >= 1
