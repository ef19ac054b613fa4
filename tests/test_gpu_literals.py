"""GPU parity of the literal find_iter engine (iter_spec_lit_kernel, used
when the regex is a finite string set): chunked find_iter over long
haystacks and over sharded spans must equal the oracle's find_iter
(re_trait.rs:197-221) bit for bit, including overlapping candidates
(`aa` in runs of `a`), priority between a literal and its prefix
(`a|ab`, `ab|a`) and matches across unit cuts."""
import random
import zlib

import numpy as np
import pytest

import regex_amd as R
from golden_data import corpus, known_counts
from oracle_py import OracleRegex
from regex_amd.dist import find_iter_spans_local

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def literal_engine(knobs):
    # force the literal engine (by default it runs only where the DFA does not
    # fit LDS exactly)
    knobs(lit=1)

PATTERNS = [r"agggtaaa|tttaccct", r"[cgt]gggtaaa|tttaccc[acg]", r"a|ab", r"ab|a", r"aa", r"e", r"(?i)holm",
            r"Sherlock|Holmes|Watson", r"foo(bar)?", r"x(a|ab)(c|bcd)", r"[0-3]{2}", r"abc|abd|ab", r"é"]


def dev(buf, cuda):
    import torch
    t = torch.zeros(len(buf) + 16, dtype=torch.uint8)
    t[: len(buf)] = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy())
    return t.to(cuda)


def pairs(m):
    return [(int(a), int(b)) for a, b in m.cpu().numpy()]


def texts(pat):
    rng = random.Random(zlib.crc32(pat.encode()))
    alpha = [b"a", b"b", b"c", b"d", b"x", b"g", b"t", b"foo", b"bar", b"0", b"1", b"2", b"3", "é".encode(),
             b"Holm", b"holm", b" ", b"aaaaaaaa"]
    yield corpus("sherlock")[:300000]
    yield corpus("regexdna")
    yield b"a" * 100001
    yield b"".join(rng.choice(alpha) for _ in range(60000))


@pytest.mark.parametrize("pat", PATTERNS)
def test_literal_find_iter(cuda, pat):
    re = R.Regex(pat)
    assert re.literals(), pat
    o = OracleRegex(re)
    for t in texts(pat):
        exp = o.find_iter(t)
        c, m = re.find_iter_batch(dev(t, cuda), stride=len(t), length=len(t), count=1)
        assert int(c[0]) == len(exp) and pairs(m) == exp, (pat, len(t))


@pytest.mark.parametrize("pat", [r"aa", r"a|ab", r"agggtaaa|tttaccct", r"Sherlock|Holmes|Watson"])
def test_literal_spans(cuda, pat):
    re = R.Regex(pat)
    o = OracleRegex(re)
    for t in texts(pat):
        exp = o.find_iter(t)
        for k in (2, 7):
            got, _ = find_iter_spans_local(re, dev(t, cuda), len(t), k)
            assert pairs(got) == exp, (pat, k)


def test_literal_batch_of_haystacks(cuda):
    re = R.Regex(r"Holmes|Watson")
    o = OracleRegex(re)
    text = corpus("sherlock")
    L = 20000
    n = len(text) // L
    buf = text[: n * L]
    c, m = re.find_iter_batch(dev(buf, cuda), stride=L, length=L, count=n)
    got, k = pairs(m), 0
    for i in range(n):
        exp = o.find_iter(buf[i * L:(i + 1) * L])
        assert int(c[i]) == len(exp) and got[k:k + len(exp)] == exp, i
        k += len(exp)


def test_regexdna_variants_literal_engine(cuda):
    kc = known_counts()["regexdna"]
    seq = R.Regex(kc["strip"]).replace_all(corpus("regexdna"), b"")
    big = seq * 50
    d = dev(big, cuda)
    for v in kc["variants"]:
        re = R.Regex(v["re"])
        c, m = re.find_iter_batch(d, stride=len(big), length=len(big), count=1)
        assert pairs(m) == OracleRegex(re).find_iter(big), v["re"]


def test_default_dispatch_large_word_set(cuda, knobs):
    """A 40-word alternation (DFA > 255 states): the literal engine is the
    default engine here; same matches as the oracle and as the DFA."""
    knobs()
    text = corpus("sherlock")
    words = sorted(set(w for w in text.decode("latin-1").split() if w.isalpha() and 6 <= len(w) <= 10))[:40]
    re = R.Regex("|".join(words))
    assert re.literals() and re.dfa_info(2)["states"] > 255
    exp = OracleRegex(re).find_iter(text)
    c, m = re.find_iter_batch(dev(text, cuda), stride=len(text), length=len(text), count=1)
    assert pairs(m) == exp
    knobs(lit=0)
    c, m = re.find_iter_batch(dev(text, cuda), stride=len(text), length=len(text), count=1)
    assert pairs(m) == exp


def test_literal_ragged_and_start(cuda):
    """Ragged batches (one unit per haystack) and a search start > 0 (look-
    behind context kept, rure.h:186-192) through the literal engine."""
    import torch
    text = corpus("sherlock")
    rng = random.Random(11)
    hs = []
    for _ in range(300):
        a = rng.randint(0, len(text) - 2000)
        hs.append(text[a:a + rng.randint(0, 2000)])
    offs = np.zeros(len(hs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(h) for h in hs])
    buf = dev(b"".join(hs), cuda)
    for pat in (r"Holmes|Watson|the", r"aa", r"a|ab"):
        re = R.Regex(pat)
        o = OracleRegex(re)
        c, m = re.find_iter_batch(buf, offsets=torch.from_numpy(offs).to(cuda))
        got, k = pairs(m), 0
        for i, h in enumerate(hs):
            exp = o.find_iter(h)
            assert int(c[i]) == len(exp) and got[k:k + len(exp)] == exp, (pat, i)
            k += len(exp)
    t = text[:200000]
    for pat in (r"Holmes|Watson|the", r"aa"):
        re = R.Regex(pat)
        o = OracleRegex(re)
        for start in (1, 5, 777):
            exp = []
            p, lm = start, None
            while p <= len(t):  # the iteration of re_trait.rs:197-221 from `start`
                mm = o.find(t, p)
                if mm is None:
                    break
                s, e = mm
                if s == e:
                    p = e + 1
                    if lm == e:
                        continue
                else:
                    p = e
                lm = e
                exp.append((s, e))
            c, m = re.find_iter_batch(dev(t, cuda), stride=len(t), length=len(t), count=1, start=start)
            assert pairs(m) == exp, (pat, start)


# ---------------------------------------------------------------------------
# find / is_match batches through the literal engine (lit_find_kernel,
# MatchType::Literal: exec.rs:601-625, 1148-1166): the leftmost start, and
# there the first literal in priority order, bit-equal to the oracle's
# leftmost-first find (the restated reference DFA) per haystack; strided and
# offset batches, start > 0, haystacks shorter than the shortest literal,
# matches at the very end of a haystack and odd lengths.
def _haystacks(pat, n, maxlen, seed):
    rng = random.Random(seed ^ zlib.crc32(pat.encode()))
    alpha = [b"a", b"b", b"c", b"d", b"x", b"g", b"t", b"foo", b"bar", b"0", b"1", b"2", b"3", "é".encode(),
             b"Holm", b"holm", b" ", b"aaaaaaaa", b"Sherlock", b"Watson", b"agggtaaa", b"tttaccct", b"\xff"]
    out = []
    for i in range(n):
        k = rng.randrange(0, maxlen)
        s = b"".join(rng.choice(alpha) for _ in range(k))[:k]
        out.append(s)
    return out


def _offsets_batch(hs, cuda):
    import torch
    offs = np.zeros(len(hs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(h) for h in hs])
    buf = b"".join(hs)
    return buf, offs, dev(buf, cuda), torch.from_numpy(offs).to(cuda)


@pytest.mark.parametrize("pat", PATTERNS)
def test_literal_find_batch_offsets(cuda, pat):
    from regex_amd import _native as NN
    re = R.Regex(pat)
    o = OracleRegex(re)
    hs = _haystacks(pat, 3000, 200, 1)
    buf, offs, dbuf, doffs = _offsets_batch(hs, cuda)
    for start in (0, 3):
        got = re.find_batch(dbuf, offsets=doffs, start=start).cpu().numpy().astype(np.uint64)
        assert NN.rure_amd_last_fwd_path() == -3
        exp = [o.find(h, start) if start <= len(h) else None for h in hs]
        for i, (h, e) in enumerate(zip(hs, exp)):
            g = None if got[i, 0] == np.uint64(2**64 - 1) else (int(got[i, 0]), int(got[i, 1]))
            assert g == e, (pat, i, h, start)
        m = re.is_match_batch(dbuf, offsets=doffs, start=start).cpu().numpy()
        assert [bool(x) for x in m] == [e is not None for e in exp], (pat, start)


@pytest.mark.parametrize("pat", [r"Sherlock|Holmes|Watson", r"a|ab", r"agggtaaa|tttaccct", r"aa"])
def test_literal_find_batch_strided(cuda, pat):
    re = R.Regex(pat)
    o = OracleRegex(re)
    L, S = 333, 336
    hs = _haystacks(pat, 5000, L, 2)
    rows = [h[:L].ljust(L, b"z") for h in hs]
    buf = b"".join(r.ljust(S, b"\0") for r in rows)
    got = re.find_batch(dev(buf, cuda), stride=S, length=L, count=len(rows)).cpu().numpy().astype(np.uint64)
    exp, _ = o.find_batch(np.frombuffer(buf, dtype=np.uint8).copy(), S, L, len(rows), nthreads=4)
    assert np.array_equal(got, exp.astype(np.uint64)), pat
    m = re.is_match_batch(dev(buf, cuda), stride=S, length=L, count=len(rows)).cpu().numpy()
    assert np.array_equal(m, o.is_match_batch(np.frombuffer(buf, dtype=np.uint8).copy(), S, L, len(rows), 4)), pat


@pytest.mark.parametrize("nwords", [3, 64])
def test_literal_find_default_dispatch(cuda, knobs, nwords):
    """Without the lit knob a set of at most 8 literals takes the literal
    engine and a larger one the DFA (measured faster there); lit=0
    (the DFA) gives the same answers, and both equal the oracle."""
    from regex_amd import _native as NN
    knobs()
    text = corpus("sherlock")
    if nwords == 3:
        pat = r"Sherlock|Holmes|Watson"
    else:
        words = sorted(set(w for w in text.decode("latin-1").split() if w.isalpha() and 5 <= len(w) <= 12))
        rng = np.random.default_rng(11)
        pat = "|".join(rng.choice(words, nwords, replace=False))
    re = R.Regex(pat)
    L = 256  # below the small-batch split (dispatch.cpp long_batch: >= 512 B)
    n = len(text) // L
    buf = text[: n * L]
    d = dev(buf, cuda)
    got = re.find_batch(d, stride=L, length=L, count=n).cpu().numpy()
    path = NN.rure_amd_last_fwd_path()
    gm = re.is_match_batch(d, stride=L, length=L, count=n).cpu().numpy()
    assert (path == -3) == (nwords <= 8), path
    assert NN.rure_amd_last_fwd_path() == path
    assert len(re.literals()) == nwords
    knobs(lit=0)
    ref = re.find_batch(d, stride=L, length=L, count=n).cpu().numpy()
    assert NN.rure_amd_last_fwd_path() != -3
    assert np.array_equal(got, ref)
    assert np.array_equal(gm, re.is_match_batch(d, stride=L, length=L, count=n).cpu().numpy())
    exp, _ = R_oracle_find(re, buf, L, n)
    assert np.array_equal(got.astype(np.uint64), exp)
    assert (got[:, 0] >= 0).sum() > n // 8


def R_oracle_find(re, buf, L, n):
    o = OracleRegex(re)
    exp, st = o.find_batch(np.frombuffer(buf, dtype=np.uint8).copy(), L, L, n, nthreads=4)
    return exp.astype(np.uint64), st
