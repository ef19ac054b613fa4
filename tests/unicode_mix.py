"""Haystack mutators for parity tests: non-ASCII and invalid UTF-8 bytes.

The tile kernel's LDS hot table holds only the ASCII-reachable states; any
byte that leaves them (a Unicode `\\d` digit such as U+0660..0669 or
U+FF10..FF19, a multi-byte `\\w` letter, a stray byte >= 0x80) sends the
16-byte chunk through the sentinel redo on the global u16 table
(dfa_scan.hip).  These helpers plant such bytes into the date-recipe batches
(regex_amd/workloads.py) at seeded positions, including across 16- and
128-byte boundaries, so that branch is compared with the oracle.
"""
import numpy as np


def _digits(rng, k, kind):
    out = []
    for _ in range(k):
        d = int(rng.integers(0, 10))
        if kind == 0:
            out.append(chr(0x0660 + d))
        elif kind == 1:
            out.append(chr(0xFF10 + d))
        else:
            out.append(str(d))
    return "".join(out)


def _token(rng):
    """One non-ASCII token (UTF-8 bytes)."""
    t = int(rng.integers(0, 9))
    mix = lambda k: "".join(_digits(rng, 1, int(rng.integers(0, 3))) for _ in range(k))
    if t == 0:   # Unicode-digit date, one digit system
        kind = int(rng.integers(0, 2))
        return (_digits(rng, 4, kind) + "-" + _digits(rng, 2, kind) + "-" + _digits(rng, 2, kind)).encode()
    if t == 1:   # date mixing ASCII, Arabic-Indic and fullwidth digits
        return (mix(4) + "-" + mix(2) + "-" + mix(2)).encode()
    if t == 2:   # almost-date: one non-digit in the middle
        return (mix(4) + "-" + mix(1) + "é-" + mix(2)).encode()
    if t == 3:   # Unicode word characters around an '@' (email pattern)
        return "café@straße.жур".encode()
    if t == 4:
        return "über@مثال.اختبار".encode()
    if t == 5:   # invalid UTF-8: lone continuation / lead bytes
        return bytes(int(x) for x in rng.integers(0x80, 0x100, size=int(rng.integers(1, 6))))
    if t == 6:   # truncated multi-byte digit before an ASCII date tail
        return b"\xd9" + b"2017-12-30"
    if t == 7:   # overlong / surrogate encodings (invalid) next to digits
        return b"\xc0\xb1\xed\xa0\x80" + b"1234-56-78"
    return "xéß中@yé.zß".encode()


def unicode_mix(buf, n, stride, length, seed, per_hay=3, frac=0.5):
    """Plant `per_hay` non-ASCII tokens into a `frac` of the n haystacks of a
    fixed-stride host batch (in place); returns the indices touched."""
    rng = np.random.default_rng(seed)
    touched = np.sort(rng.choice(n, size=int(n * frac), replace=False))
    for i in touched:
        base = int(i) * stride
        for _ in range(per_hay):
            tok = _token(rng)
            if len(tok) >= length:
                continue
            # bias positions to straddle 16-byte chunk and 128-byte tile edges
            if rng.integers(0, 2):
                edge = 16 * int(rng.integers(1, max(2, length // 16)))
                pos = edge - int(rng.integers(1, len(tok) + 1))
            else:
                pos = int(rng.integers(0, length - len(tok) + 1))
            pos = max(0, min(pos, length - len(tok)))
            buf[base + pos: base + pos + len(tok)] = np.frombuffer(tok, dtype=np.uint8)
    return touched
