"""GPU parity of the chunked find_iter for regexes with look-around
assertions (iter_scan.hip, FwdDfaDev::looks) against the oracle's sequential
find_iter (re_trait.rs:197-221 over exec.rs:632-662), bit-exact.

The reverse scan of each search runs over text[p..e] and reads p as the
text's start (exec.rs:651-661), so these cases stress what the chunked
iteration must reproduce: units whose first reverse scan reaches their start
(repaired from the true entry), reverse NoMatches that end the iteration
(\\B at a unit start), and Unicode word boundaries whose DFA quits on
non-ASCII bytes (the quitting units are served by the wave's Pike VM:
last_fwd_path -27; tests/test_gpu_iter_wave.py).
The debug knob iter_chunk forces small units (many boundaries)."""
import os
import random
import zlib

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from golden_data import corpus, stdlib_looks_fixtures
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

ASCII_PATTERNS = [r"(?-u)\b[a-c]+\b", r"(?m)^a+", r"(?m)a+$", r"(?-u)\B[ab]+", r"(?m)^$", r"(?-u)\b",
                  r"(?-u)[a-d]*\bd", r"a+\z", r"(?-u)\B\w+", r"(?-u)\b|\B[ab]", r"(?m)^[^\n]*$",
                  r"(?-u)\bd\b|\Ba", r"(?m)(?-u)^\w*\b", r"(?-u)\B"]
UNICODE_PATTERNS = [r"\b\w+\b", r"[a-z]+ed\b", r"\bthe\b", r"\B[a-z]{2}", r"(?m)^\w+"]


def _text(seed, n, nonascii):
    rng = random.Random(seed)
    alpha = [b"a", b"b", b"c", b"d", b" ", b"\n", b"x", b"@", b"e", b"d "]
    w = [8, 6, 5, 3, 6, 3, 2, 1, 3, 2]
    if nonascii:
        alpha += ["é".encode(), b"\xff"]
        w += [1, 1]
    return b"".join(rng.choices(alpha, weights=w, k=n))[:n]


def _dev(buf, cuda):
    import torch
    return torch.from_numpy(np.frombuffer(buf + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)


def _run(re, buf, L, count, cuda, chunk, **kw):
    with R.debug(iter_chunk=chunk, **kw):
        counts, m = re.find_iter_batch(_dev(buf, cuda), stride=L, length=L, count=count)
        return counts.cpu().numpy().tolist(), [tuple(x) for x in m.cpu().numpy().tolist()], N.rure_amd_last_fwd_path()


def _check(re, buf, L, count, cuda, chunk, **kw):
    o = OracleRegex(re)
    counts, got, path = _run(re, buf, L, count, cuda, chunk, **kw)
    k = 0
    for i in range(count):
        exp = o.find_iter(buf[i * L:(i + 1) * L])
        assert counts[i] == len(exp), (i, chunk)
        assert got[k:k + len(exp)] == exp, (i, chunk)
        k += len(exp)
    assert k == len(got)
    return path


@pytest.mark.parametrize("pat", ASCII_PATTERNS)
@pytest.mark.parametrize("chunk", [16, 61, 4096])
def test_find_iter_looks_chunked(cuda, pat, chunk):
    re = R.Regex(pat)
    L = 6000
    for count, seed in ((1, 1), (3, 2)):
        buf = _text(zlib.crc32(pat.encode()) + seed, L * count, False)
        assert _check(re, buf, L, count, cuda, chunk) in (-12, -14, -25, -27), pat


@pytest.mark.parametrize("pat", UNICODE_PATTERNS)
@pytest.mark.parametrize("nonascii", [False, True])
@pytest.mark.parametrize("wave", [1, 0])
def test_find_iter_unicode_boundary(cuda, pat, nonascii, wave):
    """A DFA that can quit (Unicode \\b): ASCII text stays chunked; with
    non-ASCII bytes the units whose searches quit are served by the wave's
    Pike VM inside the chunked iteration (-27); knob iter_wave=0 reads the
    quit back and sends the batch to the wave path (-13)."""
    re = R.Regex(pat)
    L = 8000
    buf = _text(zlib.crc32(pat.encode()), L, nonascii)
    path = _check(re, buf, L, 1, cuda, 64, iter_wave=wave)
    if not nonascii:
        assert path in (-12, -14, -25, -27), pat
    elif "\\b" in pat or "\\B" in pat:
        assert path == (-27 if wave else -13), pat


@pytest.mark.parametrize("pat", [r"\b\w+\b", r"(?m)^\w+", r"\bthe\b", r"(?-u:\b)[A-Z]\w*", r"\w+ing\b"])
def test_find_iter_looks_long_sherlock(cuda, pat):
    """The default unit size over ~1 MB of English (ASCII)."""
    text = corpus("sherlock")
    text = bytes(b if b < 0x80 else 0x20 for b in text)
    text = (text * 3)[:1 << 20]
    re = R.Regex(pat)
    import torch
    counts, m = re.find_iter_batch(_dev(text, cuda), stride=len(text), length=len(text), count=1)
    assert N.rure_amd_last_fwd_path() in (-12, -14, -25, -27), pat
    exp = OracleRegex(re).find_iter(text)
    assert [tuple(x) for x in m.cpu().numpy().tolist()] == exp
    del torch


@pytest.mark.parametrize("pat", stdlib_looks_fixtures()[0]["patterns"])
@pytest.mark.parametrize("chunk", [64, 4096])
def test_find_iter_looks_vs_stdlib(cuda, pat, chunk):
    """The chunked path against Python's `re` (gen_stdlib_looks.py): an
    anchor independent of the product's compiler."""
    fx, text = stdlib_looks_fixtures()
    re = R.Regex(pat)
    for (off, n), exp in zip(fx["slices"], fx["find_iter"][pat]):
        counts, got, path = _run(re, text[off:off + n], n, 1, cuda, chunk)
        assert got == [tuple(x) for x in exp], (pat, off)
        assert path in (-12, -14, -25, -27), pat


@pytest.mark.parametrize("pat", [r"\w+", r"\w+\s+\w+", r"[\w.]+@\w+", r"\pL+", r"\w{2,4}", r"(?m)^\w+",
                                 r"(?m)\w+$", r"(?m)^\pL+\s"])
@pytest.mark.parametrize("nonascii", [False, True])
@pytest.mark.parametrize("sync", [0, 1])
def test_find_iter_ascii_shadow(cuda, pat, nonascii, sync):
    """Unicode classes: the find_iter automaton's ASCII shadow (all-rows LDS
    tables, non-ASCII bytes quit) answers ASCII text; a non-ASCII byte makes
    the full automaton answer.  By default the quit stays on the device and
    gates both passes, enqueued one after the other (last_fwd_path -25);
    knob shadow_sync=1 reads it back (-14 the shadow answered, -15 the full
    automaton re-ran)."""
    re = R.Regex(pat)
    L = 20000
    buf = _text(zlib.crc32(pat.encode()) + 5, L * 2, nonascii)
    path = _check(re, buf, L, 2, cuda, 64, shadow_sync=sync)
    # (-19: the run engine of a C+ regex, which decodes UTF-8 and never quits)
    if not sync:
        assert path in (-25, -19), (pat, path)
    else:
        # (after a quit a look-around regex notes its own chunked path, -12)
        assert path in ((-15, -12, -19) if nonascii else (-14, -19)), (pat, path)
