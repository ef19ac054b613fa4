"""Host-side simulation of the exported dense DFA tables, mirroring the
kernel's algorithm (regex_amd/csrc/kernels/dfa_scan.hip) step for step.
TEST INFRASTRUCTURE: validates the eager materializer + minimiser on CPU."""


def word(b):
    return b == 0x5F or 0x30 <= b <= 0x39 or 0x41 <= b <= 0x5A or 0x61 <= b <= 0x7A


def fwd_flag(t, at):
    start, end = at == 0, len(t) == 0
    sl = at == 0 or t[at - 1] == 0x0A
    wl = at > 0 and word(t[at - 1])
    wn = at < len(t) and word(t[at])
    return (1 if start else 0) | (2 if end else 0) | (4 if sl else 0) | (8 if end else 0) | \
        (16 if wl != wn else 32) | (64 if wl else 0)


def rev_flag(t, lo, at):
    start, end = at == len(t), lo == len(t)
    sl = at == len(t) or t[at] == 0x0A
    wl = at < len(t) and word(t[at])
    wn = at > lo and word(t[at - 1])
    return (1 if start else 0) | (2 if end else 0) | (4 if sl else 0) | (8 if end else 0) | \
        (16 if wl != wn else 32) | (64 if wl else 0)


class QuitError(Exception):
    pass


def find(fwd, rev, t, start=0, mode="find", cut=None):
    """cut: the search may not start a match at or after `cut` (the kernel's
    dfa_find_cut: the state at cut - 1 is replaced by its stripped copy)."""
    info, tr, eof, st = fwd
    s = int(st[fwd_flag(t, start)])
    last = None
    if s >= info["normal"]:
        return None
    at = start
    done = False
    strip_at = cut - 1 if (cut is not None and cut > start and cut - 1 <= len(t)) else None
    while at < len(t):
        if at == strip_at:
            s = int(info["strip"][s])
            if s == info["dead"]:
                done = True
                break
        s = int(tr[s, t[at]])
        if s >= info["normal"]:
            if s < info["match_end"]:
                last = at
                if mode != "find":
                    done = True
                    break
            elif s == info["dead"]:
                done = True
                break
            else:
                raise QuitError()
        at += 1
    if not done and strip_at == len(t):
        s = int(info["strip"][s])
        done = s == info["dead"]
    if not done and eof[s]:
        last = len(t)
    if mode == "shortest":
        return last
    if mode == "is_match":
        return last is not None
    if last is None:
        return None
    if last == start:
        return (start, start)
    rinfo, rtr, reof, rst = rev
    s = int(rst[rev_flag(t, start, last)])
    rs = None
    a = last
    dead = False
    while a > start:
        a -= 1
        s = int(rtr[s, t[a]])
        if s >= rinfo["normal"]:
            if s < rinfo["match_end"]:
                rs = a + 1
            elif s == rinfo["dead"]:
                dead = True
                break
            else:
                raise QuitError()
    if not dead and reof[s]:
        rs = start
    if rs is None:  # exec.rs:656-660: the reverse DFA over text[start..] found no start -> NoMatch
        return None
    return (rs, last)


def set_matches(tables, t, start=0):
    """The set kernel's walk (dfa_scan.hip dfa_set_kernel): OR of the now
    masks of the states entered, plus the EOF mask of the last state."""
    info, tr, eof, now, st = tables
    if start > len(t):
        return 0
    s = int(st[fwd_flag(t, start)])
    mask = 0
    full = (1 << info["n"]) - 1
    if s == info["dead"]:
        return 0
    for at in range(start, len(t)):
        s = int(tr[s, t[at]])
        if s >= info["normal"]:
            if s < info["match_end"]:
                mask |= int(now[s])
                if mask == full:
                    return mask
            elif s == info["dead"]:
                return mask
            else:
                raise QuitError()
    return mask | int(eof[s])
