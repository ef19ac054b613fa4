"""The C-ABI library loads without a GPU and exports every function
include/rure_amd.h declares (no compute calls here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "rure_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(rure_\w+)\s*\(", src))
    return sorted(names)


def test_all_declared_symbols_exported():
    import regex_amd._native as N
    names = declared()
    assert len(names) >= 38
    missing = [n for n in names if not hasattr(N.lib, n)]
    assert not missing, missing


def test_error_and_options_calls_need_no_gpu():
    import regex_amd._native as N
    err = N.rure_error_new()
    assert N.rure_compile(b"(", 1, 0, None, err) is None
    assert b"unclosed" in N.rure_error_message(err).lower() or len(N.rure_error_message(err)) > 0
    N.rure_error_free(err)
    o = N.rure_options_new()
    N.rure_options_size_limit(o, 1 << 20)
    N.rure_options_free(o)
