"""GPU parity of batched find_iter (iter_scan.hip) against the oracle's
sequential find_iter (re_trait.rs:197-221), bit-exact, plus the regex-dna
known answers (examples/regexdna-output.txt) computed on the GPU."""
import random
import zlib

import numpy as np
import pytest

import regex_amd as R
from golden_data import corpus, known_counts
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

CHUNK_PATTERNS = [r"\w+", r"[a-z]+ing", r"(?i)holmes|watson", r"\w+@\w+\.\w+", r"x*", r"(?s).", r"e",
                  r"[a-q][^u-z]{13}x", r"\d+", r"(a|ab)(c|bcd)(d*)"]
WAVE_PATTERNS = [r"\b\w+\b", r"(?m)^\w+", r"\bthe\b", r"\B", r"(?-u:\b)[A-Z]\w*"]


def to_dev(buf, cuda):
    import torch
    return torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy()).to(cuda)


def as_pairs(m):
    return [(int(a), int(b)) for a, b in m.cpu().numpy()]


@pytest.mark.parametrize("pat", CHUNK_PATTERNS + WAVE_PATTERNS)
def test_find_iter_one_long_haystack(cuda, pat):
    text = corpus("sherlock")[:400000]
    re = R.Regex(pat)
    exp = OracleRegex(re).find_iter(text)
    counts, m = re.find_iter_batch(to_dev(text + b"\0" * 16, cuda), stride=len(text), length=len(text), count=1)
    assert int(counts[0]) == len(exp)
    assert as_pairs(m) == exp


@pytest.mark.parametrize("pat", CHUNK_PATTERNS[:6] + WAVE_PATTERNS[:2])
def test_find_iter_fixed_batch(cuda, pat):
    text = corpus("sherlock")
    n, L = 64, 9000
    buf = text[: n * L]
    re = R.Regex(pat)
    o = OracleRegex(re)
    counts, m = re.find_iter_batch(to_dev(buf, cuda), stride=L, length=L, count=n)
    got, k = as_pairs(m), 0
    for i in range(n):
        exp = o.find_iter(buf[i * L:(i + 1) * L])
        assert int(counts[i]) == len(exp), (pat, i)
        assert got[k:k + len(exp)] == exp, (pat, i)
        k += len(exp)
    assert k == len(got)


@pytest.mark.parametrize("pat", [r"\w+", r"a|b", r"\bo", r"x*"])
def test_find_iter_ragged_batch(cuda, pat):
    import torch
    rng = random.Random(zlib.crc32(pat.encode()))
    text = corpus("sherlock")
    hs = []
    for _ in range(500):
        a = rng.randint(0, len(text) - 300)
        hs.append(text[a:a + rng.randint(0, 300)])
    offs = np.zeros(len(hs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(h) for h in hs])
    re = R.Regex(pat)
    o = OracleRegex(re)
    counts, m = re.find_iter_batch(to_dev(b"".join(hs) + b"\0" * 16, cuda), offsets=torch.from_numpy(offs).to(cuda))
    got, k = as_pairs(m), 0
    for i, h in enumerate(hs):
        exp = o.find_iter(h)
        assert int(counts[i]) == len(exp)
        assert got[k:k + len(exp)] == exp
        k += len(exp)


def test_regexdna_known_answers(cuda):
    """examples/regexdna-output.txt: strip headers/newlines, then count variants."""
    kc = known_counts()["regexdna"]
    raw = corpus("regexdna")
    assert len(raw) == kc["input_len"]
    strip = R.Regex(kc["strip"])
    counts, m = strip.find_iter_batch(to_dev(raw + b"\0" * 16, cuda), stride=len(raw), length=len(raw), count=1)
    spans = m.cpu().numpy()
    keep = np.ones(len(raw), dtype=bool)
    for a, b in spans:
        keep[a:b] = False
    seq = np.frombuffer(raw, dtype=np.uint8)[keep].tobytes()
    assert len(seq) == kc["stripped_len"]
    dseq = to_dev(seq + b"\0" * 16, cuda)
    for v in kc["variants"]:
        c, _ = R.Regex(v["re"]).find_iter_batch(dseq, stride=len(seq), length=len(seq), count=1)
        assert int(c[0]) == v["count"], v["re"]


def test_regexdna_replicated_counts(cuda):
    """Many copies in one haystack (the C3 shape, scaled down): counts scale
    with the copies, boundaries between chunks included."""
    kc = known_counts()["regexdna"]
    raw = corpus("regexdna")
    copies = 40
    big = raw * copies
    strip = R.Regex(kc["strip"])
    o = OracleRegex(strip)
    c, m = strip.find_iter_batch(to_dev(big + b"\0" * 16, cuda), stride=len(big), length=len(big), count=1)
    assert as_pairs(m) == o.find_iter(big)


FB_PATTERNS = [r">[^\n]*\n|\n", r"a+", r"a[^b]*b", r"[ab]c*", r"\n", r">[^\n]*", r"(?-u)>[^\n]*\n|\n",
               r"a(b|cd)*e?", r"(?s)a.*b|c"]


def _fb_text(seed, n, nonascii):
    rng = random.Random(seed)
    alpha = [b"a", b"b", b"c", b"d", b"e", b"\n", b">", b"g", b"t"] + ([b"\xc3\xa9", b"\xff", b"\x80"] if nonascii else [])
    w = [8, 3, 5, 3, 2, 2, 1, 20, 20] + ([1, 1, 1] if nonascii else [])
    return b"".join(rng.choices(alpha, weights=w, k=n))


@pytest.mark.parametrize("pat", FB_PATTERNS)
@pytest.mark.parametrize("nonascii", [False, True])
def test_find_iter_first_byte_rule(cuda, pat, nonascii):
    """The first-byte start rule of the speculative pass (no reverse scan where
    the host proved the match start is the first F byte) against the oracle,
    on one long chunked haystack with ASCII-only and mixed bytes."""
    re = R.Regex(pat)
    assert re.first_bytes()
    text = _fb_text(zlib.crc32(pat.encode()), 300000, nonascii)
    exp = OracleRegex(re).find_iter(text)
    counts, m = re.find_iter_batch(to_dev(text + b"\0" * 16, cuda), stride=len(text), length=len(text), count=1)
    assert int(counts[0]) == len(exp)
    assert as_pairs(m) == exp


LEX_PATTERNS = [r">[^\n]*\n|\n", r"\n", r"a[^b]*b", r"(?-u)>[^\n]*\n|\n", r'"[^"]*"', r"<[^>]*>"]


def _lex_text(seed, n, nonascii):
    rng = random.Random(seed)
    alpha = [b"a", b"b", b"c", b"g", b"t", b"\n", b">", b'"', b"<", b" "] + ([b"\xc3\xa9", b"\xff"] if nonascii else [])
    w = [6, 2, 3, 20, 20, 2, 1, 1, 1, 3] + ([0.02, 0.02] if nonascii else [])
    return b"".join(rng.choices(alpha, weights=w, k=n))


@pytest.mark.parametrize("pat", LEX_PATTERNS)
@pytest.mark.parametrize("nonascii", [False, True])
def test_find_iter_lexer(cuda, pat, nonascii):
    """The lexer engine (iter_spec_lex_tile_kernel + tail pass) against the
    oracle and against the burst kernel (debug knob lex=0): one long haystack
    (many units) and a fixed-stride batch of several haystacks."""
    import os
    re = R.Regex(pat)
    assert re.lex_table() is not None
    o = OracleRegex(re)
    text = _lex_text(zlib.crc32(pat.encode()), 400000, nonascii)
    d = to_dev(text + b"\0" * 16, cuda)
    exp = o.find_iter(text)
    counts, m = re.find_iter_batch(d, stride=len(text), length=len(text), count=1)
    assert as_pairs(m) == exp
    with R.debug(lex=0):
        _, m0 = re.find_iter_batch(d, stride=len(text), length=len(text), count=1)
    assert as_pairs(m0) == exp
    n, L = 6, 60000
    counts, m = re.find_iter_batch(d, stride=L, length=L - 5, count=n)
    got, k = as_pairs(m), 0
    for i in range(n):
        e = o.find_iter(text[i * L:i * L + L - 5])
        assert got[k:k + len(e)] == e, (pat, i)
        k += len(e)
    assert k == len(got)


@pytest.mark.parametrize("pat", LEX_PATTERNS)
def test_find_iter_lexer_variants(cuda, pat):
    """The byte-per-step lexer (debug knob lex4=0: the fallback when the
    four-byte table does not build) gives the default path's matches; the
    default (four bytes per step) is checked against the oracle, with a
    capacity that cuts the output inside a unit."""
    import os
    re = R.Regex(pat)
    o = OracleRegex(re)
    text = _lex_text(zlib.crc32(pat.encode()) + 7, 300000, True)
    d = to_dev(text + b"\0" * 16, cuda)
    exp = o.find_iter(text)
    _, m = re.find_iter_batch(d, stride=len(text), length=len(text), count=1)
    assert as_pairs(m) == exp
    if len(exp) > 10:
        _, mc = re.find_iter_batch(d, stride=len(text), length=len(text), count=1, capacity=len(exp) // 2 + 3)
        assert as_pairs(mc)[:len(exp) // 2 + 3] == exp[:len(exp) // 2 + 3]
    with R.debug(lex4=0):
        re1 = R.Regex(pat)  # (a fresh regex: device tables keep the knobs of their first use)
        _, m1 = re1.find_iter_batch(d, stride=len(text), length=len(text), count=1)
    assert as_pairs(m1) == exp
