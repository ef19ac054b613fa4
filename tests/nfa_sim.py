"""Host-side simulation of the Pike VM kernel (regex_amd/csrc/kernels/
nfa_scan.hip) over the exported closure tables, step for step (the 64-lane
ballots become ordered loops).  TEST INFRASTRUCTURE: validates the closure
tables (host/nfa_build.cpp) and the kernel's algorithm on CPU against the
reference's golden vectors and the oracle Pike VM."""
import os
import re as _re

_HERE = os.path.dirname(os.path.abspath(__file__))
NO_CHAR = None

LK_START_LINE, LK_END_LINE, LK_START_TEXT, LK_END_TEXT = 1, 2, 4, 8
LK_WB, LK_NWB, LK_WB_ASCII, LK_NWB_ASCII = 16, 32, 64, 128


def _perlw():
    src = open(os.path.join(_HERE, "..", "oracle", "unicode_word.h")).read()
    body = src[src.index("{", src.index("ORC_PERLW")) + 1:]
    body = body[: body.index("}")]
    nums = [int(x, 16) for x in _re.findall(r"0x[0-9a-fA-F]+", body)]
    return [(nums[i], nums[i + 1]) for i in range(0, len(nums), 2)]


_PERLW = None


def unicode_word(c):
    global _PERLW
    if c is None:
        return False
    if c < 0x80:
        return ascii_word(c)
    if _PERLW is None:
        _PERLW = _perlw()
    lo, hi = 0, len(_PERLW)
    while lo < hi:
        mid = (lo + hi) // 2
        if c < _PERLW[mid][0]:
            hi = mid
        elif c > _PERLW[mid][1]:
            lo = mid + 1
        else:
            return True
    return False


def ascii_word(c):
    return c == 0x5F or 0x30 <= c <= 0x39 or 0x41 <= c <= 0x5A or 0x61 <= c <= 0x7A


def dec_utf8(s):
    if not s:
        return None
    b0 = s[0]
    if b0 <= 0x7F:
        return b0
    if 0xC0 <= b0 <= 0xDF:
        if len(s) < 2 or s[1] & 0xC0 != 0x80:
            return None
        cp = ((b0 & 0x1F) << 6) | (s[1] & 0x3F)
        return None if cp < 0x80 or cp > 0x7FF else cp
    if 0xE0 <= b0 <= 0xEF:
        if len(s) < 3 or s[1] & 0xC0 != 0x80 or s[2] & 0xC0 != 0x80:
            return None
        cp = ((b0 & 0x0F) << 12) | ((s[1] & 0x3F) << 6) | (s[2] & 0x3F)
        return None if cp < 0x800 or 0xD800 <= cp <= 0xDFFF else cp
    if 0xF0 <= b0 <= 0xF7:
        if len(s) < 4 or any(x & 0xC0 != 0x80 for x in s[1:4]):
            return None
        cp = ((b0 & 0x07) << 18) | ((s[1] & 0x3F) << 12) | ((s[2] & 0x3F) << 6) | (s[3] & 0x3F)
        return None if cp < 0x10000 or cp > 0x10FFFF else cp
    return None


def utf8_len(cp):
    return 1 if cp < 0x80 else 2 if cp < 0x800 else 3 if cp < 0x10000 else 4


def dec_last_utf8(s):
    n = len(s)
    if n == 0:
        return None
    start = n - 1
    if s[start] <= 0x7F:
        return s[start]
    lim = n - 4 if n >= 4 else 0
    while start > lim:
        start -= 1
        if s[start] & 0xC0 != 0x80:
            break
    cp = dec_utf8(s[start:])
    if cp is None or utf8_len(cp) < n - start:
        return None
    return cp


def look_holds(t, pos, info):
    if info["looks"] == 0:
        return 0
    n = len(t)
    h = 0
    if pos == 0 or t[pos - 1] == 0x0A:
        h |= LK_START_LINE
    if pos == n or t[pos] == 0x0A:
        h |= LK_END_LINE
    if pos == 0:
        h |= LK_START_TEXT
    if pos == n:
        h |= LK_END_TEXT
    ap = pos > 0 and ascii_word(t[pos - 1])
    an = pos < n and ascii_word(t[pos])
    h |= LK_WB_ASCII if ap != an else LK_NWB_ASCII
    if info["unicode_wb"]:
        wp = unicode_word(dec_last_utf8(t[:pos]))
        wn = unicode_word(dec_utf8(t[pos:]) if pos < n else None)
        h |= LK_WB if wp != wn else LK_NWB
    return h


class NfaSim(object):
    def __init__(self, tables, single):
        self.info, self.leaves, self.cl_off, self.ent = tables
        self.single = single
        self.leaves = [tuple(int(x) for x in r) for r in self.leaves]
        self.ent = [(int(a), int(b)) for a, b in self.ent]
        self.cl_off = [int(x) for x in self.cl_off]

    def append(self, cid, holds, stv, lst, members):
        o0, o1 = self.cl_off[cid], self.cl_off[cid + 1]
        for k in range(o0, o1):
            leaf, cp = self.ent[k]
            ok = (cp & 0xFF) & ~holds == 0
            pv = cp >> 8
            while ok and pv:
                q = self.ent[o0 + pv - 1][1]
                if (q & 0xFF) & ~holds == 0:
                    ok = False
                pv = q >> 8
            if ok and leaf not in members:
                members.add(leaf)
                lst.append((leaf, stv))

    def run(self, t, start=0, mode="find"):
        """mode: find -> (s, e) | None; is_match -> bool; shortest -> e | None; set -> mask."""
        info = self.info
        full = (1 << info["nmatch"]) - 1
        if start > len(t):
            return 0 if mode == "set" else (False if mode == "is_match" else None)
        clist, cmem = [], set()
        matched = all_matched = False
        mask = 0
        ms = me = None
        at = start
        while True:
            if not clist and ((matched and self.single) or all_matched or (at != 0 and info["anchored"])):
                break
            if not clist or (not info["anchored"] and not all_matched):
                self.append(info["root"], look_holds(t, at, info), at, clist, cmem)
            b = t[at] if at < len(t) else 0x100
            hnx = look_holds(t, at + 1, info) if at < len(t) else 0
            nlist, nmem = [], set()
            quit_now = False
            for leaf, stv in clist:
                w0, cid, slot = self.leaves[leaf]
                kind, lo, hi = w0 & 0xFF, (w0 >> 8) & 0xFF, (w0 >> 16) & 0xFF
                if kind == 1:
                    if mode == "set":
                        if slot < 64:
                            mask |= 1 << slot
                        matched = True
                        all_matched = all_matched or (mask & full) == full
                        if self.single:
                            break
                        continue
                    ms, me = stv, at
                    matched = all_matched = True
                    if mode != "find":
                        quit_now = True
                    break
                if lo <= b <= hi:
                    self.append(cid, hnx, stv, nlist, nmem)
            if quit_now or at >= len(t):
                break
            at += 1
            clist, cmem = nlist, nmem
        if mode == "set":
            return mask
        if mode == "is_match":
            return matched
        if mode == "shortest":
            return me
        return (ms, me) if me is not None else None


def next_utf8(t, i):
    """utf8.rs:24-39"""
    if i >= len(t):
        return i + 1
    b = t[i]
    return i + (1 if b <= 0x7F else 2 if b <= 0xDF else 3 if b <= 0xEF else 4)


class CapsSim(NfaSim):
    """The captures kernel (nfa_scan.hip caps_kernel / pike_caps): thread
    lists carry slot rows; an entry's Saves set its slots to the add position."""

    def __init__(self, tables, saves, nslots):
        NfaSim.__init__(self, tables, True)
        self.save_off = [int(x) for x in saves[0]]
        self.save_slot = [int(x) for x in saves[1]]
        self.ns = nslots

    def append_caps(self, cid, holds, prow, at, lst, members):
        o0, o1 = self.cl_off[cid], self.cl_off[cid + 1]
        for k in range(o0, o1):
            leaf, cp = self.ent[k]
            ok = (cp & 0xFF) & ~holds == 0
            pv = cp >> 8
            while ok and pv:
                q = self.ent[o0 + pv - 1][1]
                if (q & 0xFF) & ~holds == 0:
                    ok = False
                pv = q >> 8
            if ok and leaf not in members:
                members.add(leaf)
                row = list(prow) if prow is not None else [None] * self.ns
                for q in range(self.save_off[k], self.save_off[k + 1]):
                    if self.save_slot[q] < self.ns:
                        row[self.save_slot[q]] = at
                lst.append((leaf, row))

    def pike(self, t, start):
        """Slots of the leftmost-first match in t from start, or None."""
        info = self.info
        if start > len(t):
            return None
        out = None
        clist, cmem = [], set()
        at = start
        while True:
            if not clist and (out is not None or (at != 0 and info["anchored"])):
                break
            if not clist or (not info["anchored"] and out is None):
                self.append_caps(info["root"], look_holds(t, at, info), None, at, clist, cmem)
            b = t[at] if at < len(t) else 0x100
            hnx = look_holds(t, at + 1, info) if at < len(t) else 0
            nlist, nmem = [], set()
            for leaf, row in clist:
                w0, cid, _ = self.leaves[leaf]
                kind, lo, hi = w0 & 0xFF, (w0 >> 8) & 0xFF, (w0 >> 16) & 0xFF
                if kind == 1:
                    out = list(row)
                    break
                if lo <= b <= hi:
                    self.append_caps(cid, hnx, row, at + 1, nlist, nmem)
            if at >= len(t):
                break
            at += 1
            clist, cmem = nlist, nmem
        if out is None or out[0] is None or out[1] is None:
            return None
        return out

    def captures(self, t, start, bounds):
        """caps_kernel's dispatch given the DFA's bounds: (s, e) -> Pike VM
        from s over t[..min(next_utf8(next_utf8(e)), len)]; None -> no match;
        "quit" (or an anchored program) -> the whole text from start."""
        if not self.info["anchored"] and bounds != "quit":
            if bounds is None:
                return None
            s, e = bounds
            return self.pike(t[:min(next_utf8(t, next_utf8(t, e)), len(t))], s)
        return self.pike(t, start)
