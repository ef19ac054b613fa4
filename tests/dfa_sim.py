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


def find(fwd, rev, t, start=0, mode="find", cut=None, fb=None, out=None):
    """cut: the search may not start a match at or after `cut` (the kernel's
    dfa_find_cut: the state at cut - 1 is replaced by its stripped copy).
    fb: the first-byte start rule's bytes (iter_scan.hip, host
    first_byte_rule): when the scan ended in the dead state and every byte it
    read was ASCII, the start is the first fb byte at or after `start`.
    out: a dict; out["reached"] says the reverse scan reached `start` alive
    (its answer then depends on where the search began: the slice quirk)."""
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
        if out is not None:
            out["reached"] = True
        return (start, start)
    if fb and done and all(b < 0x80 for b in t[start:at + 1]):
        return (next(i for i in range(start, last) if t[i] in fb), last)
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
    if out is not None:
        out["reached"] = not dead
    if out is not None:
        out["stop"] = rs is None  # a NoMatch that ends the reference's iteration
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


def core_set_matches(tables, t, start=0, n=64):
    """The core-form set kernel's walk (dfa_scan.hip set_core_kernel): chunks
    of 16 bytes through the hot table with an output bag, redone against the
    global tables when they leave the hot cores or meet output code 63."""
    info, cls, T, gcore, gout, eof, st, masktab = tables
    hot, dead, quit = info["hot"], info["dead"], info["quit"]
    full = (1 << n) - 1 if n < 64 else (1 << 64) - 1
    if start > len(t):
        return 0
    c = int(st[fwd_flag(t, start)])
    mask = 0
    if c == dead:
        return 0

    def careful(c, mask, b):
        k = int(cls[b])
        mask |= int(gout[c, k])
        c = int(gcore[c, k])
        if c == quit:
            raise QuitError()
        return c, mask, c == dead or (mask & full) == full

    def step1(c, mask, b):
        k = int(cls[b])
        if c < hot:
            e = int(T[c, k])
            code = e & 63
            if (e >> 6) != hot and code != 63:
                if code:
                    mask |= int(masktab[code])
                c = e >> 6
                if c == quit:
                    raise QuitError()
                return c, mask, c == dead or (mask & full) == full
        return careful(c, mask, b)

    at = start
    done = False
    while not done and at < len(t) and (at % 16) != 0:  # haystack base is 16-aligned here
        c, mask, done = step1(c, mask, t[at])
        at += 1
    while not done and at + 16 <= len(t):
        chunk = t[at:at + 16]
        ok = False
        if c < hot:
            x, bag, pend = c, 0, 0
            for b in chunk:
                e = int(T[x, int(cls[b])])
                bag |= 1 << (e & 63)
                if (e & 63) == 63:
                    pend |= int(gout[x, int(cls[b])])
                x = e >> 6
            if x != hot:
                for code in range(1, 63):  # codes 1..62: the code mask table
                    if (bag >> code) & 1:
                        mask |= int(masktab[code])
                mask |= pend
                c = x
                if c == quit:
                    raise QuitError()
                done = c == dead or (mask & full) == full
                ok = True
        if not ok:
            for b in chunk:
                c, mask, done = careful(c, mask, b)
                if done:
                    break
        at += 16
    while not done and at < len(t):
        c, mask, done = step1(c, mask, t[at])
        at += 1
    if not done:
        mask |= int(eof[c])
    return mask
