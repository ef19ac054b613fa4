"""GPU parity of the Shift-And find_iter engine (iter_spec_sa_kernel, the
default for string sets whose strings all have one length, e.g. the
regex-dna variants): chunked find_iter over long haystacks, sharded spans,
batches of fixed-stride and ragged haystacks and a search start > 0 must
equal the oracle's find_iter (re_trait.rs:197-221) bit for bit — including
self-overlapping strings (`aa` in runs of `a`, `agggtaaa` after `agg`),
strings merged into class sequences (`(?i)holm`, `[0-3]{2}`), multi-byte
UTF-8 strings, and matches across unit cuts.  Each case runs through the
coalesced tile kernel (the default for fixed-stride batches of whole
128-byte-line units), the per-lane kernel (knob sa=2) and the DFA burst
kernel (sa=0)."""
import random
import zlib

import numpy as np
import pytest

import regex_amd as R
from golden_data import corpus, known_counts
from oracle_py import OracleRegex
from regex_amd.dist import find_iter_spans_local

pytestmark = pytest.mark.gpu

# every pattern is a set of strings of one length (the engine's domain)
PATTERNS = [r"agggtaaa|tttaccct", r"[cgt]gggtaaa|tttaccc[acg]", r"agggt[cgt]aa|tt[acg]accct", r"aa", r"e",
            r"(?i)holm", r"Holmes|Watson", r"[0-3]{2}", r"abc|abd", r"é", r"x(ab|cd)y", r"aaaaaaa"]


def dev(buf, cuda):
    import torch
    t = torch.zeros(len(buf) + 16, dtype=torch.uint8)
    t[: len(buf)] = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy())
    return t.to(cuda)


def pairs(m):
    return [(int(a), int(b)) for a, b in m.cpu().numpy()]


def texts(pat):
    rng = random.Random(zlib.crc32(pat.encode()))
    alpha = [b"a", b"b", b"c", b"d", b"x", b"y", b"g", b"t", b"0", b"1", b"2", b"3", "é".encode(), b"Holm",
             b"holm", b"HOLM", b" ", b"aaaaaaaa", b"agggtaaa", b"tttaccct", b"agg", b"xaby", b"xcdy"]
    yield corpus("sherlock")[:300000]
    yield corpus("regexdna")
    yield b"a" * 100001
    yield b"".join(rng.choice(alpha) for _ in range(60000))


def both_engines(knobs):
    # default (coalesced tile kernel where the batch allows it), the per-lane
    # Shift-And kernel (knob sa=2), the DFA burst kernel (sa=0)
    for v in (None, 2, 0):
        if v is None:
            knobs()
        else:
            knobs(sa=v)
        yield v


@pytest.mark.parametrize("pat", PATTERNS)
def test_shiftand_find_iter(cuda, pat, knobs):
    re = R.Regex(pat)
    lits = re.literals()
    assert lits and len(set(len(x) for x in lits)) == 1, pat
    o = OracleRegex(re)
    for t in texts(pat):
        exp = o.find_iter(t)
        d = dev(t, cuda)
        for _ in both_engines(knobs):
            c, m = re.find_iter_batch(d, stride=len(t), length=len(t), count=1)
            assert int(c[0]) == len(exp) and pairs(m) == exp, (pat, len(t))


@pytest.mark.parametrize("pat", [r"aa", r"agggtaaa|tttaccct", r"Holmes|Watson", r"aaaaaaa"])
def test_shiftand_spans(cuda, pat):
    re = R.Regex(pat)
    o = OracleRegex(re)
    for t in texts(pat):
        exp = o.find_iter(t)
        for k in (2, 7, 64):
            got, _ = find_iter_spans_local(re, dev(t, cuda), len(t), k)
            assert pairs(got) == exp, (pat, k)


def test_shiftand_batches_and_start(cuda):
    import torch
    text = corpus("sherlock")
    re = R.Regex(r"Holmes|Watson")
    o = OracleRegex(re)
    L = 20000
    n = len(text) // L
    buf = text[: n * L]
    c, m = re.find_iter_batch(dev(buf, cuda), stride=L, length=L, count=n)
    got, k = pairs(m), 0
    for i in range(n):
        exp = o.find_iter(buf[i * L:(i + 1) * L])
        assert int(c[i]) == len(exp) and got[k:k + len(exp)] == exp, i
        k += len(exp)
    rng = random.Random(5)
    hs = []
    for _ in range(300):
        a = rng.randint(0, len(text) - 2000)
        hs.append(text[a:a + rng.randint(0, 2000)])
    offs = np.zeros(len(hs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(h) for h in hs])
    d = dev(b"".join(hs), cuda)
    for pat in (r"Holmes|Watson", r"aa", r"(?i)the"):
        re = R.Regex(pat)
        o = OracleRegex(re)
        c, m = re.find_iter_batch(d, offsets=torch.from_numpy(offs).to(cuda))
        got, k = pairs(m), 0
        for i, h in enumerate(hs):
            exp = o.find_iter(h)
            assert int(c[i]) == len(exp) and got[k:k + len(exp)] == exp, (pat, i)
            k += len(exp)
    t = text[:200000]
    for pat in (r"Holmes|Watson", r"aa"):
        re = R.Regex(pat)
        o = OracleRegex(re)
        # every start, including inside a match of the whole-text iteration
        straddling = [s + 1 for s, e in o.find_iter(t)[:3] if e - s > 1]
        for start in [1, 777, 100003] + straddling:
            c, m = re.find_iter_batch(dev(t, cuda), stride=len(t), length=len(t), count=1, start=start)
            assert pairs(m) == o.find_iter(t, start), (pat, start)


def test_regexdna_variants_shiftand(cuda):
    kc = known_counts()["regexdna"]
    seq = R.Regex(kc["strip"]).replace_all(corpus("regexdna"), b"")
    big = seq * 50
    d = dev(big, cuda)
    for v in kc["variants"]:
        re = R.Regex(v["re"])
        c, m = re.find_iter_batch(d, stride=len(big), length=len(big), count=1)
        got = pairs(m)
        assert got == OracleRegex(re).find_iter(big), v["re"]
        assert len(got) == 50 * v["count"] + 49 * (len(OracleRegex(re).find_iter(seq * 2)) - 2 * v["count"])


@pytest.mark.parametrize("L", [70001, 70003, 4099])
def test_shiftand_haystack_end(cuda, L, knobs):
    """Odd-length haystacks followed, inside their stride, by bytes that would
    complete a match straddling the end: the kernels read whole aligned
    16-byte blocks (include/rure_amd.h: the buffer must be readable to its
    16-byte-rounded end) but take no byte past the haystack's end."""
    import torch
    n, S = 8, (L + 16 + 15) & ~15
    rng = random.Random(L)
    buf = bytearray()
    for i in range(n):
        body = bytes(rng.choice(b"acgt") for _ in range(L - 5)) + b"agggt"   # a match cut at the end
        buf += body + b"aaa" + b"agggtaaa"[: S - L - 3].ljust(S - L - 3, b"a")
    d = torch.from_numpy(np.frombuffer(bytes(buf), dtype=np.uint8).copy()).to(cuda)
    re = R.Regex(r"agggtaaa|tttaccct")
    o = OracleRegex(re)
    for _ in both_engines(knobs):
        c, m = re.find_iter_batch(d, stride=S, length=L, count=n)
        got, k = pairs(m), 0
        for i in range(n):
            exp = o.find_iter(bytes(buf[i * S:i * S + L]))
            assert int(c[i]) == len(exp) and got[k:k + len(exp)] == exp, (L, i)
            k += len(exp)
