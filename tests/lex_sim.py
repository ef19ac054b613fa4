"""Host-side simulation of iter_spec_lex_tile_kernel (iter_scan.hip): the
lexer table walk with the per-block flag words, the first-byte start
positions recovered from them, and the hand-over to the generic cut-bounded
iteration for a unit's last byte.
TEST INFRASTRUCTURE: validates the lexer algorithm on CPU."""
NONE = None


def lex16(lex, s, blk, kend):
    """One 16-byte block on the byte table (iter_scan.hip lex16): returns the
    flag word (2 bits per byte) and the entry after the block."""
    tab, _ = lex
    m = 0
    for k in range(kend):
        s = int(tab[76 * s + blk[k]])
        m |= (s & 3) << (2 * k)
    return m, s


LEX4_FLAGS, LEX4_CLS = 2048, 4096  # dfa_scan.hpp kLex4Flags, kLex4Cls


def lex16x4(lex4, s, blk, kend):
    """The same block four bytes per step (iter_scan.hip lex16x4, host
    build_lex4): s is a row; bytes from kend on take class 3 (no byte)."""
    tab, _ = lex4
    m = 0
    for j in range(4):
        c = 0
        for k in range(4):
            i = 4 * j + k
            c |= 3 << (2 * k) if i >= kend else int(tab[LEX4_CLS + 256 * k + blk[i]])
        a = (s << 8) | c
        m |= int(tab[LEX4_FLAGS + a]) << (8 * j)
        s = int(tab[a])
    return m, s


def lex_walk(lex, t, c0, end):
    """Walk text[c0, end) from the start state as the kernel does, block by
    block (16-byte blocks aligned to c0 here), the events of two blocks at a
    time (lex_events).  A block holding a byte >= 0x80 freezes the walk (the
    kernel leaves the rest to the tail pass).  Returns (matches, p, lm,
    frozen, hint): the matches whose search ended inside, the iteration
    state after them, whether the walk froze, and the tail pass's scan-from
    hint."""
    tab, s0 = lex
    s = s0
    cz = 1                 # the state before c0 is the start state
    fc = None
    p, lm = c0, NONE
    out = []
    frozen = False
    blocks = []            # (bp, m) of the pair being collected
    bp = c0

    def events(b0, m0, m1):
        nonlocal cz, fc, p, lm
        M = m0 | (m1 << 32)
        E = (M >> 1) & 0x5555555555555555
        Z = (M ^ (M >> 1)) & 0x5555555555555555
        A = (E | (Z << 2) | cz) & 0xFFFFFFFFFFFFFFFF
        while E:
            j = (E & -E).bit_length() - 1
            E &= E - 1
            below = A & ((1 << j) - 1)
            f = b0 + (below.bit_length() - 1) // 2 if below else fc
            x = b0 + j // 2
            out.append((f, x))
            p = lm = x
        if A:
            fc = b0 + (A.bit_length() - 1) // 2
        cz = (Z >> 62) & 1

    while bp < end:
        kend = min(16, end - bp)
        if any(b >= 0x80 for b in t[bp:bp + kend]):
            frozen = True
            break
        m, s = lex16(lex, s, t[bp:bp + kend], kend)
        blocks.append((bp, m))
        if len(blocks) == 2:
            events(blocks[0][0], blocks[0][1], blocks[1][1])
            blocks = []
        bp += 16
    if blocks:  # a pair's first block alone (its second was not lexed)
        events(blocks[0][0], blocks[0][1], 0)
    return out, p, lm, frozen, max(p, fc if fc is not None else c0)


def lex_unit(tab, fwd, rev, t, c0, c1):
    """One unit's speculative iteration as the kernel computes it: the lexer
    over [c0, min(c1 - 1, len)) up to a block holding a byte >= 0x80, then the
    tail pass's generic cut-bounded iteration from the state it left.
    Returns (matches, exit, clean)."""
    from iter_sim import UnitIter
    ms, p, lm, _, fc = lex_walk(tab, t, c0, max(c0, min(c1 - 1, len(t))))
    it = UnitIter(fwd, rev, t, (p, lm), c1, scan_from=fc)
    while True:
        m = it.next()
        if m is None:
            break
        ms.append(m)
    return ms, it.exit, it.clean
