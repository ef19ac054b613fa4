"""The one-byte-class replace_all (rure_amd_replace_batch without a match
list, replace_scan.hip launch_replace_class): which regexes qualify (host
class_one_set, read off the syntax tree) — every byte the class holds must
be a whole match of the regex and no other byte a match start (checked
against the oracle byte by byte) — and which must not (multi-byte matches,
case-insensitive literals, Unicode classes beyond ASCII, repetitions)."""
import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex

CLASS_PATS = [r"B", r"[KM]", r"(?-u)\xff", r"[a-c]", r"x", r"(?-u)\w", r"(?s-u:.)", r"[\n]", r"(?-u:.)", r"(B)",
              r"(?:[0-9])", r"\x00"]
NOT_CLASS = [r"(?i)k", r"ab", r"é", r"\w", r".", r"B+", r"", r"[a-c]?", r"\bB", r"B|CD", r"(?s:.)"]


def class_of(pat):
    c = np.zeros(256, dtype=np.uint8)
    re = R.Regex(pat)  # (held: the handle is freed with the object)
    return c if N.rure_amd_class_one_export(re._re, c.ctypes.data) == 1 else None


@pytest.mark.parametrize("pat", CLASS_PATS)
def test_class_one_exact(pat):
    cls = class_of(pat)
    assert cls is not None, pat
    o = OracleRegex(R.Regex(pat))
    for b in range(256):
        t = bytes([b])
        assert (o.find_iter(t) == [(0, 1)]) == bool(cls[b]), (pat, b)
        # a class byte between two others is its own match
        t3 = b"\x01" + t + b"\x02"
        ms = o.find_iter(t3)
        assert ((1, 2) in ms) == bool(cls[b]), (pat, b)


@pytest.mark.parametrize("pat", NOT_CLASS)
def test_not_class_one(pat):
    assert class_of(pat) is None, pat
