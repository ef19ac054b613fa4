"""Host-side simulation of the chunked find_iter pipeline of
regex_amd/csrc/kernels/iter_scan.hip (speculative units, lockstep repair,
sequential walker, emit), over the exported find_iter DFA tables.
TEST INFRASTRUCTURE: validates the boundary-repair algorithm on CPU."""
from dfa_sim import QuitError, find

NONE = None
STOP = float("inf")  # the exit of an iteration that ended (a search's NoMatch)


def wave_search(nfa):
    """iter_scan.hip iter_next with a WaveCtx (the wave-served units of a
    regex with a Unicode word boundary): a search whose DFA quits runs on the
    NFA (nfa(t, start): the reference's NFA search, exec.rs:485-487) bounded
    by the cut; a search from just after a byte >= 0x80 that finds no match
    before the cut runs the DFA unbounded, as the reference does, and takes
    the NFA's answer if that scan quits (its start flags read the byte as a
    non-word byte, dfa.rs:1423)."""
    def search(fwd, rev, t, start=0, mode="find", cut=None, fb=None, out=None):
        def by_nfa():
            if out is not None:
                out["reached"] = False
            m = nfa(t, start)
            if m is None or (cut is not None and start < cut and m[0] >= cut):
                return None
            return tuple(m)
        try:
            m = find(fwd, rev, t, start, mode, cut, fb, out)
        except QuitError:
            return by_nfa()
        if m is None and start > 0 and t[start - 1] >= 0x80 and cut is not None and start < cut:
            try:
                find(fwd, rev, t, start, mode, None, fb, {})
            except QuitError:
                return by_nfa()
        return m
    return search


class UnitIter(object):
    def __init__(self, fwd, rev, t, st, c1, fb=None, scan_from=0, search=find):
        self.fwd, self.rev, self.t, self.fb = fwd, rev, t, fb
        self.search = search
        self.p, self.lm = st
        self.c1 = c1
        # the first search may scan from here (no match starts in [p, scan_from):
        # the lexer's hand-over to the tail pass, iter_lex_tail_kernel)
        self.scan_from = scan_from
        self.ended = False
        self.clean = False
        self.exit = None
        # the first search's reverse scan reached the entry alive: with
        # look-around its answer depends on where the search began (the
        # reverse slice starts there, dfa_sim.find), so a speculation entered
        # fresh is not equivalent to the true iteration entering earlier
        self.unsure = False
        self.first = True
        self.stop = False

    def _iter_next(self):
        t = self.t
        while True:
            if self.p > len(t):
                return None
            out = {}
            m = self.search(self.fwd, self.rev, t, self.p, cut=self.c1, fb=self.fb, out=out)
            if self.first:
                self.unsure = out.get("reached", False)
                self.first = False
            if m is None:
                # the reverse scan found no start (look-around at the slice
                # start): the reference's iteration ends here
                self.stop = out.get("stop", False)
                return None
            s, e = m
            if s == e:
                self.p = e + 1
                if self.lm == e:
                    continue
            else:
                self.p = e
            self.lm = e
            return m

    def next(self):
        if self.ended:
            return None
        if self.p == STOP:
            self.ended, self.exit, self.clean = True, (STOP, None), False
            return None
        if self.p >= self.c1:
            self.ended = True
            self.exit = (self.p, self.lm)
            self.clean = self.p == self.c1 and self.lm != self.c1
            return None
        snap = (self.p, self.lm)
        self.p = max(self.p, self.scan_from)
        m = self._iter_next()
        if m is not None and m[0] < self.c1:
            return m
        self.p, self.lm = snap
        self.ended = True
        self.exit = snap
        self.clean = True
        if m is None and self.stop:
            self.exit, self.clean = (STOP, None), False
        return None


def equiv(ca, a, cb, b, strict=False):
    """two unit exits lead the next unit alike: both clean (a fresh start at
    its c0) or the same state; strict (the next unit's speculation is unsure)
    takes only the same state"""
    if strict:
        return a == b
    if ca or cb:
        return ca and cb
    return a == b


def find_iter_chunked(fwd, rev, t, chunk, start=0, slots=1 << 30, fb=None, looks=False, nfa=None):
    """nfa: the wave-served iteration of a regex with a Unicode word
    boundary (wave_search; a unit after a byte >= 0x80 is unsure)."""
    INF = float("inf")
    search = wave_search(nfa) if nfa else find
    span = max(0, len(t) - start)
    nk = 1 if span <= chunk else (span + chunk - 1) // chunk
    bounds = [(start + k * chunk, INF if k + 1 == nk else start + (k + 1) * chunk) for k in range(nk)]
    units = []
    for k, (c0, c1) in enumerate(bounds):  # pass 1: speculation
        it = UnitIter(fwd, rev, t, (c0, None), c1, fb, search=search)
        ms = []
        while True:
            m = it.next()
            if m is None:
                break
            ms.append(m)
        units.append({"entry": (c0, None), "spec": ms, "spec_exit": it.exit, "spec_clean": it.clean,
                      "unsure": k > 0 and ((looks and it.unsure) or (nfa is not None and t[c0 - 1] >= 0x80)),
                      "exit": it.exit, "clean": it.clean, "fixed": False, "count": len(ms)})

    def sync_from_slots(j, E):
        """repair_unit's fast path: S's recorded matches tell where the true
        iteration entered with E joins the speculative one."""
        c0, c1 = bounds[j]
        U = units[j]
        spec = U["spec"]
        if looks or len(spec) > slots or E[0] < c0:
            return None
        # p_i, lm_i: S's iteration state before it yielded match i
        ps, lms = [c0], [None]
        for (s_, e_) in spec:
            ps.append(e_ + 1 if s_ == e_ else e_)
            lms.append(e_)
        i = max(k for k in range(len(ps)) if ps[k] <= E[0])
        if E[0] == ps[i] and E[1] != lms[i]:
            # same search start, different last match: S's search from p_i
            # yielded its match i directly (no empty match skipped) when it
            # had no last match (i == 0) or match i starts at p_i
            if not (i == 0 or (i < len(spec) and spec[i][0] == ps[i])):
                return None
        if i < len(spec):
            s_, e_ = spec[i]
            if s_ < E[0] or (s_ == e_ and e_ == E[1]):
                return None
            return i
        return i if U["spec_clean"] else None

    def strict(j):
        return j + 1 < nk and units[j + 1]["unsure"]

    def repair(j, E):
        c0, c1 = bounds[j]
        U = units[j]
        U["entry"], U["fixed"], U["skip"] = E, True, None
        if E[0] >= c1:  # the true iteration skips the whole unit
            U["count"], U["exit"] = 0, E
            U["clean"] = E[0] == c1 and E[1] != c1
            return not equiv(U["clean"], U["exit"], U["spec_clean"], U["spec_exit"], strict(j))
        i = sync_from_slots(j, E)
        if i is not None:
            if i < len(U["spec"]):
                U["count"], U["skip"] = len(U["spec"]) - i, i
                U["exit"], U["clean"] = U["spec_exit"], U["spec_clean"]
                return False
            U["count"], U["exit"], U["clean"] = 0, E, True
            return not equiv(True, E, U["spec_clean"], U["spec_exit"], strict(j))
        F = UnitIter(fwd, rev, t, E, c1, search=search)
        S = UnitIter(fwd, rev, t, (c0, None), c1, search=search)
        fm, sm = F.next(), S.next()
        fcnt = scnt = 0
        synced = False
        while fm is not None:
            if sm is not None and fm == sm:
                synced = True
                break
            if sm is None or fm < sm:
                fcnt += 1
                fm = F.next()
            else:
                scnt += 1
                sm = S.next()
        if synced:
            U["count"] = fcnt + U_len(U) - scnt
            if fcnt == 0 and len(U["spec"]) <= slots:
                U["skip"] = scnt
            U["exit"], U["clean"] = U["spec_exit"], U["spec_clean"]
            return False
        U["count"] = fcnt
        changed = not equiv(F.clean, F.exit, U["spec_clean"], U["spec_exit"], strict(j))
        U["exit"], U["clean"] = F.exit, F.clean
        return changed

    def U_len(U):
        return len(U["spec"])

    queue = []
    for u in range(nk - 1):  # pass 2: parallel repair
        if not units[u]["spec_clean"] or units[u + 1]["unsure"]:
            if repair(u + 1, units[u]["spec_exit"]):
                queue.append(u + 1)
    walked = 0  # pass 3: sequential walker
    for j in sorted(queue):
        if j + 1 <= walked:
            continue
        u = j + 1
        X = units[j]
        while u < nk:
            P = units[u - 1]
            if equiv(X["clean"], X["exit"], P["spec_clean"], P["spec_exit"], strict(u - 1)):
                break
            if X["clean"] and not units[u]["unsure"]:
                W = units[u]
                W["entry"], W["exit"], W["clean"], W["fixed"], W["count"], W["skip"] = \
                    (bounds[u][0], None), W["spec_exit"], W["spec_clean"], False, len(W["spec"]), None
            else:
                repair(u, X["exit"])
            X = units[u]
            u += 1
        walked = u
    out = []  # pass 4: emit
    for u, U in enumerate(units):
        if U["count"] == 0:
            continue
        if not U["fixed"]:
            assert len(U["spec"]) == U["count"]
            out.extend(U["spec"])
            continue
        if U.get("skip") is not None:  # repaired by joining the speculation: copy
            out.extend(U["spec"][U["skip"]:U["skip"] + U["count"]])
            continue
        it = UnitIter(fwd, rev, t, U["entry"], bounds[u][1], search=search)
        got = []
        while len(got) < U["count"]:
            m = it.next()
            assert m is not None
            got.append(m)
        out.extend(got)
    return out
