r"""The wave-served chunked find_iter (iter_scan.hip iter_wspec_kernel ..
iter_wemit_kernel, last_fwd_path -27) against the oracle's sequential
find_iter (re_trait.rs:197-221 over exec.rs:473-514), bit-exact.

A Unicode \b makes the reference's lazy DFA quit on any byte >= 0x80
(dfa.rs:1491-1496) and that one search runs on its NFA instead
(exec.rs:485-487).  Here the lane passes of the chunked iteration run as
usual, and a unit where a search quit is taken over by one wave that runs
such searches on the Pike VM, bounded by the unit's cut; its repairs, the
walker and its re-emission run on the wave too.  Cases: sparse and dense
non-ASCII bytes, tiny units (knob iter_chunk: matches spanning many units,
walker chains through wave units), several haystacks, and the VERDICT r05
workload \b\w+n\b over sherlock as it is replicated to 1 GiB (copies x 8366,
bench/src/sherlock.rs:171, plus the matches across copy seams)."""
import random
import zlib

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from golden_data import corpus, known_counts
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

PATTERNS = [r"\b\w+n\b", r"\b\w+\b", r"[a-z]+ed\b", r"\bthe\b", r"\B[a-z]{2}", r"\w+\b", r"\b\w", r"\b"]


def _dev(buf, cuda):
    import torch
    return torch.from_numpy(np.frombuffer(buf + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)


def _text(seed, n, every):
    """English-like words and separators; a non-ASCII letter or byte about
    every `every` bytes (0: none)."""
    rng = random.Random(seed)
    words = [b"the", b"then", b"when", b"seen", b"added", b"ran", b"holmes", b"a", b"in", b"on", b"x1", b"_n"]
    seps = [b" ", b" ", b", ", b".\n", b"-", b"  "]
    odd = ["é".encode(), "ñ".encode(), b"\xff", "中".encode(), "’".encode(), "ёn".encode()]
    out, k = [], 0
    while k < n:
        w = rng.choice(words)
        if every and rng.random() < 6.0 / every:
            w = w[: rng.randint(0, len(w))] + rng.choice(odd) + w[rng.randint(0, len(w)):]
        out.append(w)
        out.append(rng.choice(seps))
        k += len(w) + len(out[-1])
    return b"".join(out)[:n]


def _check(re, buf, L, count, cuda, chunk=None):
    kw = {"iter_chunk": chunk} if chunk else {}
    with R.debug(**kw):
        counts, m = re.find_iter_batch(_dev(buf, cuda), stride=L, length=L, count=count)
        path = N.rure_amd_last_fwd_path()
    got = [tuple(x) for x in m.cpu().numpy().tolist()]
    o = OracleRegex(re)
    k = 0
    for i in range(count):
        exp = o.find_iter(buf[i * L:(i + 1) * L])
        assert int(counts[i]) == len(exp), (i, chunk)
        assert got[k:k + len(exp)] == exp, (i, chunk)
        k += len(exp)
    assert k == len(got)
    return path


@pytest.mark.parametrize("pat", PATTERNS)
@pytest.mark.parametrize("every", [3000, 40])
@pytest.mark.parametrize("chunk", [16, 61, 509, 4096])
def test_wave_units_vs_oracle(cuda, pat, every, chunk):
    re = R.Regex(pat)
    L = 24000 if chunk >= 509 else 6000
    for count, seed in ((1, 1), (3, 2)):
        buf = _text(zlib.crc32(pat.encode()) + seed * 7 + every, L * count, every)
        assert _check(re, buf, L, count, cuda, chunk) == -27, pat


@pytest.mark.parametrize("pat", [r"\b\w+n\b", r"\b\w+\b"])
def test_wave_default_units(cuda, pat):
    """The default unit size over ~2 MB of sherlock as it is (33 non-ASCII
    bytes per copy) and over the same text with a non-ASCII letter every
    ~200 bytes."""
    t = corpus("sherlock")
    re = R.Regex(pat)
    t3 = (t * 4)[: 2 << 20]
    assert _check(re, t3, len(t3), 1, cuda) == -27
    a = bytearray(t3)
    for i in range(0, len(a) - 1, 199):
        if 0x61 <= a[i] <= 0x7A and 0x61 <= a[i + 1] <= 0x7A:
            a[i], a[i + 1] = 0xC3, 0xA9
    assert _check(re, bytes(a), len(a), 1, cuda) == -27


def test_wave_empty_and_tiny(cuda):
    re = R.Regex(r"\b\w+n\b")
    for buf in (b"", "é".encode(), "né n".encode(), b"\xffn n\xff", "ñn".encode() * 50):
        L = max(1, len(buf))
        b2 = buf if buf else b"\0"
        _check(re, b2[:L], L, 1, cuda, 16)


def test_wave_sherlock_one_gib(cuda):
    r"""\b\w+n\b over sherlock as it is, replicated to 1 GiB as one haystack:
    copies x 8366 (bench/src/sherlock.rs:171) plus the seam matches, the
    first copy's records equal to the oracle's (VERDICT r05 ask 4)."""
    import torch
    t = corpus("sherlock")
    e = next(x for x in known_counts()["sherlock"] if x["re"] == r"\b\w+n\b")
    assert e["count"] == 8366
    re = R.Regex(r"\b\w+n\b")
    seam = len(OracleRegex(re).find_iter(t * 2)) - 2 * e["count"]
    copies = (1 << 30) // len(t)
    one = torch.from_numpy(np.frombuffer(t, dtype=np.uint8).copy()).to(cuda)
    big = torch.zeros(copies * len(t) + 16, dtype=torch.uint8, device=cuda)
    big[:copies * len(t)].view(copies, len(t)).copy_(one.expand(copies, len(t)))
    n = copies * len(t)
    counts, m = re.find_iter_batch(big, stride=n, length=n, count=1, capacity=copies * e["count"] + copies * seam)
    assert N.rure_amd_last_fwd_path() == -27
    assert int(counts[0]) == copies * e["count"] + (copies - 1) * seam
    exp = OracleRegex(re).find_iter(t)[:e["count"] - 1]
    got = [tuple(x) for x in m[:len(exp)].cpu().numpy().tolist()]
    assert got == exp


@pytest.mark.parametrize("pat", [r"\b\w+n\b", r"\b", r"\B[a-z]{2}", r"\w+\b"])
def test_wave_ragged(cuda, pat):
    """A ragged batch (one unit per haystack): 400 haystacks of 0-2000 bytes,
    sparse and dense non-ASCII, empty ones included."""
    import torch
    rng = random.Random(zlib.crc32(pat.encode()))
    texts = [_text(rng.randrange(1 << 30), rng.choice([0, 1, 5, 64, 300, 2000]), rng.choice([0, 40, 3000]))
             for _ in range(400)]
    offs = np.zeros(len(texts) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(x) for x in texts])
    buf = torch.from_numpy(np.frombuffer(b"".join(texts) + bytes(16), dtype=np.uint8).copy()).to(cuda)
    re = R.Regex(pat)
    counts, m = re.find_iter_batch(buf, offsets=torch.from_numpy(offs).to(cuda))
    o = OracleRegex(re)
    exp = [o.find_iter(x) for x in texts]
    assert counts.cpu().numpy().tolist() == [len(x) for x in exp]
    assert [tuple(x) for x in m.cpu().numpy().tolist()] == [s for x in exp for s in x]
