"""CPU check of the find_iter run engine's premise (host run_class,
unicode_run_set, run_iter.hip): for a regex detected as one class repeated
(C+), the reference's iteration (re_trait.rs:197-221, restated by the
oracle) yields exactly the maximal runs of C bytes — over all bytes for a
byte class, over ASCII text for a class whose bytes >= 0x80 quit, and for a
Unicode class over any bytes with the kernel's UTF-8 rule (a byte is in C
when it belongs to a valid encoding of a code point of C, found from the
nearest lead byte at most three bytes back, never before the search start;
runs_utf8 below restates run_iter.hip's utf8_in_class).  Regexes that are
not C+ (lazy, bounded, anchored, look-around, sequences) must not be
detected."""
import random
import zlib

import numpy as np
import pytest

import regex_amd as R
from oracle_py import OracleRegex

RUNS = [r"\w+", r"[a-z]+", r"\S+", r"\pL+", r"\d+", r"(?-u)\w+", r"a+", r"[^\n]+", r".+", r"\s+",
        r"(?i)[a-f]+", r"(?s).+", r"[^a]+", r"[0-9A-Fa-f]+", r"(?:[a-c]|[x-z])+", r"[a-z][a-z]*", r"\w\w*"]
NOT_RUNS = [r"\w+?", r"(?:ab)+", r"a+b", r"\w{2,4}", r"\b\w+", r"(?m)^\w+", r"x*", r"[a-z]+ing", r"\w+\b",
            r"a|b+", r"[a-z]+[0-9]", r"\w{2,}", r"(?m)\w+$", r"\pL"]


def runs(cls, t):
    a = np.frombuffer(t, dtype=np.uint8)
    m = (cls[a] & 1).astype(bool)
    out, i, n = [], 0, len(t)
    while i < n:
        if m[i]:
            j = i
            while j < n and m[j]:
                j += 1
            out.append((i, j))
            i = j
        else:
            i += 1
    return out


def _utf8_at(t, lo, q, cp):
    """run_iter.hip utf8_in_class: byte q of t (bytes before lo invisible)"""
    p = q
    k = 0
    while k < 3 and p > lo and (t[p] & 0xC0) == 0x80:
        p -= 1
        k += 1
    b0 = t[p]
    if 0xC2 <= b0 <= 0xDF:
        n, c = 2, b0 & 0x1F
    elif 0xE0 <= b0 <= 0xEF:
        n, c = 3, b0 & 0x0F
    elif 0xF0 <= b0 <= 0xF4:
        n, c = 4, b0 & 0x07
    else:
        return False
    if p + n <= q or p + n > len(t):
        return False
    for i in range(1, n):
        bi = t[p + i]
        if (bi & 0xC0) != 0x80:
            return False
        if i == 1 and ((b0 == 0xE0 and bi < 0xA0) or (b0 == 0xED and bi > 0x9F) or (b0 == 0xF0 and bi < 0x90)
                       or (b0 == 0xF4 and bi > 0x8F)):
            return False
        c = (c << 6) | (bi & 0x3F)
    return bool((int(cp[c >> 5]) >> (c & 31)) & 1)


def runs_utf8(cls, cp, t, lo=0):
    """the run engine's matches from lo: maximal runs of bytes in C"""
    m = [False] * len(t)
    for q in range(lo, len(t)):
        m[q] = bool(cls[t[q]] & 1) if t[q] < 0x80 else _utf8_at(t, lo, q, cp)
    out, i = [], lo
    while i < len(t):
        if m[i]:
            j = i
            while j < len(t) and m[j]:
                j += 1
            out.append((i, j))
            i = j
        else:
            i += 1
    return out


# UTF-8 noise: letters, digits, marks, spaces, symbols, an astral letter,
# and invalid forms (a stray continuation, truncated leads, overlong, a
# surrogate, past U+10FFFF, 0xFF)
UTF8_NOISE = ["é", "ß", "Ω", "٣", "́", " ", " ", "✓", "—", "中", "𝐀", "😀", "K", "ſ"]
BAD = [b"\x80", b"\xbf", b"\xc3", b"\xe2\x80", b"\xf0\x9f\x98", b"\xc0\xaf", b"\xe0\x80\xaf", b"\xed\xa0\x80",
       b"\xf4\x90\x80\x80", b"\xff", b"\xc3\xc3\xa9"]


def utf8_text(seed, n):
    rng = random.Random(seed)
    alpha = [b"a", b"b", b"f", b"x", b"Z", b"0", b"9", b" ", b"\n", b"_", b"-"]
    alpha += [c.encode() for c in UTF8_NOISE] * 2 + BAD
    return b"".join(rng.choices(alpha, k=n))


def text(seed, n, nonascii):
    rng = random.Random(seed)
    alpha = [b"a", b"b", b"f", b"x", b"Z", b"0", b"9", b" ", b" ", b"\n", b"\t", b"_", b".", b"-", b"@"]
    if nonascii:
        alpha += ["é".encode(), "✓".encode(), b"\xff", "٣".encode()]
    return b"".join(rng.choices(alpha, k=n))[:n]


@pytest.mark.parametrize("pat", RUNS)
def test_run_class_detected_and_exact(pat):
    re = R.Regex(pat)
    cls = re.run_class()
    if cls is None:
        cls = re.run_class(ascii=True)
    assert cls is not None, pat
    o = OracleRegex(re)
    if cls[0x80] & 4:  # a Unicode class: the UTF-8 rule over any bytes
        cp = re.run_code_points()
        assert cp is not None and len(cp) == 0x110000 // 32, pat
        for i in range(6):
            t = utf8_text(zlib.crc32(pat.encode()) + i, 200 + 31 * i)
            for st in (0, 1, 2, 7):
                assert runs_utf8(cls, cp, t, st) == o.find_iter(t, st), (pat, st, t)
        return
    quits = bool(cls[0x80] & 2)
    for i in range(8):
        nonascii = not quits and i % 2 == 1
        t = text(zlib.crc32(pat.encode()) + i, 300 + 37 * i, nonascii)
        assert runs(cls, t) == o.find_iter(t), (pat, t)
        for st in (1, 5, 17):  # a search from start: runs of text[start:]
            exp = o.find_iter(t, st)
            got = [(a + st, b + st) for a, b in runs(cls, t[st:])]
            assert got == exp, (pat, st)


@pytest.mark.parametrize("pat", NOT_RUNS)
def test_not_runs(pat):
    re = R.Regex(pat)
    assert re.run_class() is None and re.run_class(ascii=True) is None, pat


UNICODE_RUNS = [r"\w+", r"\pL+", r"\S+", r"[^\n]+", r"\d+", r"(?i)[a-z]+", r"[\x80-\x{10FFFF}]+", r"\p{Greek}+",
                r"(?:\w)+", r"(\w)+", r".+", r"(?s).+"]


@pytest.mark.parametrize("pat", UNICODE_RUNS)
def test_unicode_run_code_points(pat):
    """The bitmap holds exactly the code points whose encoding the regex
    matches whole (sampled: all of U+0000..U+07FF and a stride over the rest),
    and the ASCII bytes' class bits agree with it."""
    re = R.Regex(pat)
    cp = re.run_code_points()
    assert cp is not None, pat
    cls = re.run_class()
    o = OracleRegex(re)
    cps = list(range(0x800)) + list(range(0x800, 0x110000, 997))
    for c in cps:
        if 0xD800 <= c <= 0xDFFF:
            continue
        e = chr(c).encode()
        full = o.find_iter(e) == [(0, len(e))]
        assert bool((int(cp[c >> 5]) >> (c & 31)) & 1) == full, (pat, hex(c))
        if c < 0x80:
            assert bool(cls[c] & 1) == full
    assert all(cls[b] == 4 for b in range(0x80, 0x100))


@pytest.mark.parametrize("pat", [r"(?-u)\w+", r"[a-z]+", r"\w+?", r"\w{2,}", r"\pL"])
def test_no_unicode_run(pat):
    assert R.Regex(pat).run_code_points() is None
