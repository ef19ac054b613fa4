"""The debug override table (regex_amd/csrc/host/knobs.hpp): one table, read
once per process from RURE_AMD_DEBUG and replaced as a whole through
rure_amd_debug_set; unknown names and malformed values are refused and leave
the table unchanged.  No other RURE_AMD_* variable is read by the library."""
import os
import re

import pytest

import regex_amd as R
from regex_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "regex_amd", "csrc")


def _names():
    src = open(os.path.join(CSRC, "host", "knobs.cpp")).read()
    block = src[src.index("kNames[kN] = {"):src.index("};", src.index("kNames[kN] = {"))]
    return re.findall(r'"([a-z0-9_]+)"', block)


def test_every_knob_name_accepted():
    names = _names()
    enum = open(os.path.join(CSRC, "host", "knobs.hpp")).read()
    body = enum[enum.index("enum class Knob"):enum.index("kCount")]
    assert len(names) == len(re.findall(r"^\s+[A-Z][A-Za-z0-9]*,", body, re.M))
    try:
        for n in names:
            assert N.rure_amd_debug_set(("%s=1" % n).encode()) == N.OK, n
        assert N.rure_amd_debug_set(",".join("%s=0" % n for n in names).encode()) == N.OK
    finally:
        R._debug_set(None)


@pytest.mark.parametrize("spec", ["nope=1", "lex4", "lex4=x", "lex4=-3", "lex4=1,bogus=2"])
def test_bad_specs_refused(spec):
    assert N.rure_amd_debug_set(spec.encode()) == N.ERR_ARG
    with pytest.raises(ValueError):
        R._debug_set(spec)


def test_debug_block_restores():
    R._debug_set("lex=0")
    try:
        with R.debug(lex4=0, iter_chunk=4096) as d:
            assert d.spec == "lex4=0,iter_chunk=4096"
            assert R._debug_spec[0] == d.spec
        assert R._debug_spec[0] == "lex=0"
    finally:
        R._debug_set(None)
    assert N.rure_amd_debug_set(None) == N.OK and N.rure_amd_debug_set(b"") == N.OK


def test_no_other_environment_knobs():
    """Every override goes through the table: the library reads no other
    RURE_AMD_* variable."""
    hits = []
    for d, _, files in os.walk(CSRC):
        for f in files:
            if f.endswith((".cpp", ".hpp", ".hip", ".h")):
                for m in re.finditer(r'getenv\("(RURE_AMD_[A-Z0-9_]*)"\)', open(os.path.join(d, f)).read()):
                    if m.group(1) != "RURE_AMD_DEBUG":
                        hits.append((f, m.group(1)))
    assert hits == []
