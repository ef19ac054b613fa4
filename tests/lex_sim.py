"""Host-side simulation of iter_spec_lex_tile_kernel (iter_scan.hip): the
lexer table walk with the per-block flag words, the first-byte start
positions recovered from them, and the hand-over to the generic cut-bounded
iteration for a unit's last byte.
TEST INFRASTRUCTURE: validates the lexer algorithm on CPU."""
PITCH, EMIT, Z = 264, 1, 2
NONE = None


def lex_walk(tab, t, c0, end):
    """Walk text[c0, end) from the start state as the kernel does, block by
    block (16-byte blocks aligned to c0 here).  Returns (matches, p, lm,
    nonascii): the matches whose search ended inside, the iteration state
    after them, and whether any byte was >= 0x80 (the kernel then redoes the
    unit with the generic path)."""
    flat = tab.reshape(-1)
    s = 0                  # row offset of S0
    carry_z = 1            # the state before c0 is the start state
    fc = None
    p, lm = c0, NONE
    out = []
    nonascii = any(b >= 0x80 for b in t[c0:end])
    for bp in range(c0, end, 16):
        m = 0
        kend = min(16, end - bp)
        for k in range(kend):
            e = int(flat[(s & ~7) + t[bp + k]])
            m |= (e & 3) << (2 * k)
            s = e
        E = m & 0x55555555
        zb = m & 0xAAAAAAAA & ((1 << (2 * kend - 1)) - 1)   # Z of bytes 0..kend-2
        A = E | (zb << 1) | carry_z
        while E:
            j = (E & -E).bit_length() - 1
            E &= E - 1
            below = A & ((1 << j) - 1)
            f = bp + (below.bit_length() - 1) // 2 if below else fc
            x = bp + j // 2
            out.append((f, x))
            p = lm = x
        if A:
            fc = bp + (A.bit_length() - 1) // 2
        carry_z = (m >> (2 * kend - 1)) & 1
    return out, p, lm, nonascii


def lex_unit(tab, fwd, rev, t, c0, c1, last_unit):
    """One unit's speculative iteration as the kernel computes it: the lexer
    over [c0, c1 - 1) (full units, ASCII), then the generic cut-bounded
    iteration from the state it left (the search in progress at the cut);
    ragged last units and units with non-ASCII bytes run the generic
    iteration from c0.  Returns (matches, exit, clean)."""
    from iter_sim import UnitIter
    if last_unit or c1 - 1 <= c0:
        ms, st = [], (c0, NONE)
    else:
        ms, p, lm, nonascii = lex_walk(tab, t, c0, c1 - 1)
        st = (c0, NONE) if nonascii else (p, lm)
        if nonascii:
            ms = []
    it = UnitIter(fwd, rev, t, st, c1)
    while True:
        m = it.next()
        if m is None:
            break
        ms.append(m)
    return ms, it.exit, it.clean
