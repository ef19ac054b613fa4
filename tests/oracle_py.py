"""Test-side binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE: the oracle is the checker (and bench.py's cpu_baseline),
never a product path.  It runs the reference's lazy DFA / Pike VM restatement
over the byte programs the product compiler exports.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "build", "liboracle.so")
_lib = ctypes.CDLL(LIB)
VP = ctypes.c_void_p
SZ = ctypes.c_size_t


class Stats(ctypes.Structure):
    _fields_ = [("fwd_bytes", ctypes.c_uint64), ("rev_bytes", ctypes.c_uint64),
                ("quits", ctypes.c_uint64), ("flushes", ctypes.c_uint64), ("states", ctypes.c_uint64)]


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


orc_prog_new = _sig("orc_prog_new", VP, VP, ctypes.c_uint32, ctypes.c_uint32, VP, ctypes.c_int, ctypes.c_int,
                    ctypes.c_int, ctypes.c_int, ctypes.c_uint32, SZ)
orc_regex_new = _sig("orc_regex_new", VP, VP, VP, VP)
orc_regex_free = _sig("orc_regex_free", None, VP)
orc_regex_set_exec = _sig("orc_regex_set_exec", None, VP, ctypes.c_int, ctypes.c_char_p, SZ, ctypes.c_int,
                          ctypes.c_char_p, SZ, ctypes.c_int, ctypes.c_char_p, SZ)
orc_cache_new = _sig("orc_cache_new", VP, VP)
orc_cache_free = _sig("orc_cache_free", None, VP)
orc_find_at = _sig("orc_find_at", ctypes.c_int, VP, VP, ctypes.c_char_p, SZ, SZ, ctypes.POINTER(SZ),
                   ctypes.POINTER(SZ))
orc_shortest_nfa = _sig("orc_shortest_nfa", ctypes.c_int, VP, VP, ctypes.c_char_p, SZ, SZ, ctypes.POINTER(SZ))
orc_find_nfa = _sig("orc_find_nfa", ctypes.c_int, VP, VP, ctypes.c_char_p, SZ, SZ, ctypes.POINTER(SZ),
                    ctypes.POINTER(SZ))
orc_shortest_match_at = _sig("orc_shortest_match_at", ctypes.c_int, VP, VP, ctypes.c_char_p, SZ, SZ,
                             ctypes.POINTER(SZ))
orc_is_match_at = _sig("orc_is_match_at", ctypes.c_int, VP, VP, ctypes.c_char_p, SZ, SZ)
orc_captures_nfa = _sig("orc_captures_nfa", ctypes.c_int, VP, VP, ctypes.c_char_p, SZ, SZ, VP, SZ)
orc_captures_at = _sig("orc_captures_at", ctypes.c_int, VP, VP, ctypes.c_char_p, SZ, SZ, VP, SZ)
orc_find_iter = _sig("orc_find_iter", ctypes.c_int64, VP, VP, ctypes.c_char_p, SZ, VP, SZ)
orc_find_iter_at = _sig("orc_find_iter_at", ctypes.c_int64, VP, VP, ctypes.c_char_p, SZ, SZ, VP, SZ)
orc_many_matches_at = _sig("orc_many_matches_at", ctypes.c_int, VP, VP, ctypes.c_char_p, SZ, SZ, VP)
orc_many_matches_nfa = _sig("orc_many_matches_nfa", ctypes.c_int, VP, VP, ctypes.c_char_p, SZ, SZ, VP)
orc_cache_stats = _sig("orc_cache_stats", None, VP, ctypes.POINTER(Stats))
orc_find_batch = _sig("orc_find_batch", ctypes.c_int, VP, VP, VP, SZ, SZ, SZ, ctypes.c_int, VP,
                      ctypes.POINTER(Stats))
orc_is_match_batch = _sig("orc_is_match_batch", ctypes.c_int, VP, VP, VP, SZ, SZ, SZ, ctypes.c_int, VP)
orc_shortest_batch = _sig("orc_shortest_batch", ctypes.c_int, VP, VP, VP, SZ, SZ, SZ, ctypes.c_int, VP)
orc_set_batch = _sig("orc_set_batch", ctypes.c_int, VP, VP, VP, SZ, SZ, SZ, ctypes.c_int, VP)
orc_set_batch_stats = _sig("orc_set_batch_stats", ctypes.c_int, VP, VP, VP, SZ, SZ, SZ, ctypes.c_int, VP, VP)

NONE = (1 << 64) - 1


def _prog(info_insts, dfa_size_limit=2 << 20):
    info, raw = info_insts
    bc = (ctypes.c_uint8 * 256)(*info.byte_classes)
    return orc_prog_new(raw.ctypes.data, info.ninsts, info.start, bc, info.is_reverse, info.anchored_start,
                        info.anchored_end, info.has_unicode_word_boundary, info.ncaptures, dfa_size_limit)


class OracleRegex(object):
    """Oracle over the programs of a regex_amd.Regex (or RegexSet)."""

    def __init__(self, re_obj, dfa_size_limit=2 << 20, dispatch=True):
        """dispatch: restate the reference's engine choice for a single regex
        (exec.rs:1130-1210: Literal / DfaSuffix arms, with the literal sets
        the product's host code computes); False: the DFA arms only."""
        self.is_set = hasattr(re_obj, "_set") and not hasattr(re_obj, "_re")
        if self.is_set:
            fwd = _prog(re_obj.program(0), dfa_size_limit)
            nfa = _prog(re_obj.program(2), dfa_size_limit)
            try:
                rev = _prog(re_obj.program(1), dfa_size_limit)
            except ValueError:
                rev = None
            self.n = len(re_obj)
        else:
            fwd = _prog(re_obj.program(0), dfa_size_limit)
            rev = _prog(re_obj.program(1), dfa_size_limit)
            nfa = _prog(re_obj.program(2), dfa_size_limit)
            self.ncaps = re_obj.program(2)[0].ncaptures
        self._r = orc_regex_new(nfa, fwd, rev)
        if dispatch and not self.is_set:
            import regex_amd as R
            mi = re_obj.match_info()
            pre = R._ser_lits(re_obj.exec_literals("prefixes"))
            suf = R._ser_lits(re_obj.exec_literals("suffixes"))
            self.match_type = R.MATCH_TYPES.index(mi["match_type"])
            orc_regex_set_exec(self._r, self.match_type, pre, len(pre), mi["prefix_matcher"], suf, len(suf),
                               mi["suffix_matcher"], mi["lcs"], len(mi["lcs"]))
        self._c = orc_cache_new(self._r)

    def __del__(self):
        if getattr(self, "_c", None):
            orc_cache_free(self._c)
        if getattr(self, "_r", None):
            orc_regex_free(self._r)

    def find(self, text, start=0):
        s, e = SZ(), SZ()
        if orc_find_at(self._r, self._c, text, len(text), start, ctypes.byref(s), ctypes.byref(e)):
            return (s.value, e.value)
        return None

    def find_nfa(self, text, start=0):
        s, e = SZ(), SZ()
        if orc_find_nfa(self._r, self._c, text, len(text), start, ctypes.byref(s), ctypes.byref(e)):
            return (s.value, e.value)
        return None

    def shortest_nfa(self, text, start=0):
        e = SZ()
        if orc_shortest_nfa(self._r, self._c, text, len(text), start, ctypes.byref(e)):
            return e.value
        return None

    def shortest_match(self, text, start=0):
        e = SZ()
        if orc_shortest_match_at(self._r, self._c, text, len(text), start, ctypes.byref(e)):
            return e.value
        return None

    def is_match(self, text, start=0):
        return bool(orc_is_match_at(self._r, self._c, text, len(text), start))

    def captures(self, text, start=0):
        """exec.rs:524-596 read_captures_at (the reference's dispatch)."""
        return self._caps(orc_captures_at, text, start)

    def captures_nfa(self, text, start=0):
        """Forced Pike VM over the whole text."""
        return self._caps(orc_captures_nfa, text, start)

    def _caps(self, fn, text, start):
        n = 2 * self.ncaps
        slots = np.zeros(max(n, 1), dtype=np.uint64)
        if not fn(self._r, self._c, text, len(text), start, slots.ctypes.data, n):
            return None
        out = []
        for i in range(self.ncaps):
            a, b = int(slots[2 * i]), int(slots[2 * i + 1])
            out.append(None if a == NONE or b == NONE else (a, b))
        return out

    def find_iter(self, text, start=0):
        """re_trait.rs:197-221, the first search at `start` (find_at semantics)."""
        cap = 16
        while True:
            buf = np.zeros(2 * cap, dtype=np.uint64)
            n = orc_find_iter_at(self._r, self._c, text, len(text), start, buf.ctypes.data, cap)
            if n <= cap:
                return [(int(buf[2 * i]), int(buf[2 * i + 1])) for i in range(n)]
            cap = n

    def find_iter_array(self, text, start=0, cap=None):
        """find_iter as an (n, 2) uint64 array (no per-match Python objects;
        the bench's CPU baseline).  `cap`: expected matches (rerun if short)."""
        cap = cap if cap is not None else len(text) // 32 + 1024
        while True:
            buf = np.empty(2 * max(cap, 1), dtype=np.uint64)
            n = orc_find_iter_at(self._r, self._c, text, len(text), start, buf.ctypes.data, cap)
            if n <= cap:
                return buf[: 2 * n].reshape(n, 2)
            cap = n

    def matches(self, text, start=0, nfa=False):
        m = np.zeros(max(self.n, 1), dtype=np.uint8)
        f = orc_many_matches_nfa if nfa else orc_many_matches_at
        f(self._r, self._c, text, len(text), start, m.ctypes.data)
        return [i for i in range(self.n) if m[i]]

    def stats(self):
        s = Stats()
        orc_cache_stats(self._c, ctypes.byref(s))
        return {k: getattr(s, k) for k, _ in Stats._fields_}

    # batch baselines (numpy host buffers)
    def find_batch(self, buf, stride, length, n, nthreads=1, offsets=None):
        out = np.zeros(2 * n, dtype=np.uint64)
        st = Stats()
        orc_find_batch(self._r, buf.ctypes.data, offsets.ctypes.data if offsets is not None else None,
                       stride, length, n, nthreads, out.ctypes.data, ctypes.byref(st))
        return out.reshape(n, 2), {k: getattr(st, k) for k, _ in Stats._fields_}

    def is_match_batch(self, buf, stride, length, n, nthreads=1, offsets=None):
        out = np.zeros(n, dtype=np.uint8)
        orc_is_match_batch(self._r, buf.ctypes.data, offsets.ctypes.data if offsets is not None else None,
                           stride, length, n, nthreads, out.ctypes.data)
        return out

    def shortest_batch(self, buf, stride, length, n, nthreads=1, offsets=None):
        """shortest_match end per haystack (uint64, 2**64 - 1 for none)."""
        out = np.zeros(n, dtype=np.uint64)
        orc_shortest_batch(self._r, buf.ctypes.data, offsets.ctypes.data if offsets is not None else None,
                           stride, length, n, nthreads, out.ctypes.data)
        return out

    def set_batch(self, buf, stride, length, n, nthreads=1, offsets=None, stats=False):
        out = np.zeros(n, dtype=np.uint64)
        st = Stats()
        orc_set_batch_stats(self._r, buf.ctypes.data, offsets.ctypes.data if offsets is not None else None,
                            stride, length, n, nthreads, out.ctypes.data, ctypes.byref(st))
        if stats:
            return out, {k: getattr(st, k) for k, _ in Stats._fields_}
        return out
