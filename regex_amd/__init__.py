"""regex_amd — MI355X drop-in for the batched `regex::bytes::Regex` scan path.

Python mirror of the reference's operator interface for this path
(`regex::bytes::Regex` / `RegexSet`, src/re_bytes.rs:114-623,
src/re_set.rs:86-254) over the C ABI in include/rure_amd.h.  Every search
runs on the GPU through librure_amd.so; single-haystack calls stage the
bytes to HBM, batch calls take device tensors (torch) that are already
resident.

    re = regex_amd.Regex(r"\\d{4}-\\d{2}-\\d{2}")
    re.find(b"on 2017-12-30")                     # -> (3, 13)
    starts, ends = re.find_batch(buf, stride=4096, length=4096, count=n)
"""
import ctypes

from . import _native as N

__all__ = ["Regex", "RegexSet", "Error", "NoExpand", "NONE", "release_scratch"]

NONE = N.NONE


def _ser_lits(lits):
    out = bytearray()
    for v, cut in lits:
        out += bytes([1 if cut else 0]) + len(v).to_bytes(4, "little") + bytes(v)
    return bytes(out)


def _de_lits(buf):
    out, i = [], 0
    while i < len(buf):
        cut, n = buf[i] != 0, int.from_bytes(buf[i + 1:i + 5], "little")
        out.append((bytes(buf[i + 5:i + 5 + n]), cut))
        i += 5 + n
    return out


def _call_out(fn, *args):
    n = fn(*args, None, 0)
    if n < 0:
        raise ValueError("literal extraction failed (%d)" % n)
    buf = ctypes.create_string_buffer(max(n, 1))
    fn(*args, buf, n)
    return buf.raw[:n]


def syntax_literals(pattern, which="prefixes", unicode=True, limit_size=250, limit_class=10):
    """regex-syntax's Expr::prefixes / suffixes (regex-syntax/src/literals.rs)
    of a pattern, as [(bytes, cut), ...] in the reference's order (host only)."""
    if isinstance(pattern, str):
        pattern = pattern.encode("utf-8")
    return _de_lits(_call_out(N.rure_amd_literals_syntax, pattern, len(pattern),
                              N.FLAG_UNICODE if unicode else 0, 0 if which == "prefixes" else 1,
                              limit_size, limit_class))


def literals_op(op, lits):
    """Literals::unambiguous_prefixes ("unambiguous_prefixes" / "unambiguous_suffixes",
    -> [(bytes, cut)]), longest_common_prefix / _suffix ("lcp" / "lcs" -> bytes)."""
    code = {"unambiguous_prefixes": 0, "lcp": 1, "lcs": 2, "unambiguous_suffixes": 3}[op]
    raw = _ser_lits(lits)
    out = _call_out(N.rure_amd_literals_op, code, raw, len(raw))
    return out if op in ("lcp", "lcs") else _de_lits(out)


MATCH_TYPES = ["Literal(Unanchored)", "Literal(AnchoredStart)", "Literal(AnchoredEnd)", "Dfa",
               "DfaAnchoredReverse", "DfaSuffix", "Nfa", "Nothing"]


def release_scratch():
    """Returns the device scratch the library keeps cached between batched
    calls to the allocator (rure_amd_release_scratch); also happens when the
    last Regex / RegexSet is freed."""
    N.rure_amd_release_scratch()


_debug_spec = [None]


class debug:
    """Debug-only engine overrides for a block (rure_amd_debug_set; the knob
    names are in regex_amd/csrc/host/knobs.hpp), restoring the previous
    overrides after it:

        with regex_amd.debug(lex4=0):      # the byte-per-step lexer
            ...

    For tests and A/B tools; the production dispatch never needs one.
    Tables a regex already built keep the overrides they were built under."""

    def __init__(self, **knobs):
        self.spec = ",".join("%s=%d" % (k, int(v)) for k, v in knobs.items())

    def __enter__(self):
        self.prev = _debug_spec[0]
        _debug_set(self.spec)
        return self

    def __exit__(self, *exc):
        _debug_set(self.prev)
        return False


def _debug_set(spec):
    if N.rure_amd_debug_set(spec.encode() if spec else None) != N.OK:
        raise ValueError("unknown debug knob or bad value in %r" % spec)
    _debug_spec[0] = spec


def scratch_stats():
    """{"cached", "live", "handles"}: scratch bytes cached for reuse, bytes
    held by calls in flight, rure / rure_set handles alive."""
    c, l, h = N.c_size(0), N.c_size(0), ctypes.c_long(0)
    N.rure_amd_scratch_stats(ctypes.byref(c), ctypes.byref(l), ctypes.byref(h))
    return {"cached": c.value, "live": l.value, "handles": h.value}


class Error(Exception):
    """Invalid pattern (regex-capi/src/error.rs:8-77)."""


def _flags(case_insensitive=False, multi_line=False, dot_matches_new_line=False,
           swap_greed=False, ignore_whitespace=False, unicode=True):
    f = 0
    if case_insensitive: f |= N.FLAG_CASEI
    if multi_line: f |= N.FLAG_MULTI
    if dot_matches_new_line: f |= N.FLAG_DOTNL
    if swap_greed: f |= N.FLAG_SWAP_GREED
    if ignore_whitespace: f |= N.FLAG_SPACE
    if unicode: f |= N.FLAG_UNICODE
    return f


def _options(size_limit, dfa_size_limit):
    if size_limit is None and dfa_size_limit is None:
        return None
    o = N.rure_options_new()
    if size_limit is not None:
        N.rure_options_size_limit(o, size_limit)
    if dfa_size_limit is not None:
        N.rure_options_dfa_size_limit(o, dfa_size_limit)
    return o


def _check(rc, what):
    if rc == N.OK:
        return
    names = {N.ERR_ARG: "bad argument", N.ERR_HIP: "HIP runtime error",
             N.ERR_DFA: "automaton could not be materialized"}
    raise RuntimeError("%s failed: %s (%d)" % (what, names.get(rc, "error"), rc))


def _batch(haystack, offsets=None, stride=None, length=None, count=None, start=0):
    """Describes a batch of device-resident haystacks (torch uint8 tensor)."""
    import torch
    if not isinstance(haystack, torch.Tensor) or not haystack.is_cuda:
        raise TypeError("haystack must be a torch CUDA (HIP) uint8 tensor")
    if haystack.dtype != torch.uint8 or not haystack.is_contiguous():
        raise TypeError("haystack must be a contiguous uint8 tensor")
    b = N.RureBatch()
    b.haystack = haystack.data_ptr()
    b.start = start
    if offsets is not None:
        if offsets.dtype != torch.int64 or not offsets.is_cuda or not offsets.is_contiguous():
            raise TypeError("offsets must be a contiguous int64 CUDA tensor of n+1 entries")
        b.offsets = offsets.data_ptr()
        b.count = offsets.numel() - 1
        b.stride = 0
        b.length = 0
    else:
        if stride is None or length is None:
            raise TypeError("give offsets, or stride and length")
        n = count if count is not None else (haystack.numel() // stride if stride else 0)
        if n and (n - 1) * stride + length > haystack.numel():
            raise ValueError("batch exceeds the haystack buffer")
        b.offsets = None
        b.stride = stride
        b.length = length
        b.count = n
    return b


def _stream_ptr(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class NoExpand(object):
    """A replacement used literally, `$` included (re_bytes.rs:1014-1032)."""

    def __init__(self, rep):
        self.rep = bytes(rep)


def _cap_letter(b):
    return 48 <= b <= 57 or 97 <= b <= 122 or 65 <= b <= 90 or b == 95


def _find_cap_ref(rep):
    """expand.rs:127-166: (name or number, end) of the reference at rep[0]."""
    if len(rep) <= 1 or rep[0] != 0x24:
        return None
    i, brace = 1, False
    if rep[i] == 0x7B:
        brace, i = True, 2
    end = i
    while end < len(rep) and _cap_letter(rep[end]):
        end += 1
    if end == i:
        return None
    cap = rep[i:end].decode("ascii")
    if brace:
        if end >= len(rep) or rep[end] != 0x7D:
            return None
        end += 1
    try:
        ref = int(cap)
        if ref >= 1 << 32:
            ref = cap
    except ValueError:
        ref = cap
    return ref, end


def expand(groups, names, rep, text):
    """expand.rs:50-91 (expand_bytes): `$N`, `$name`, `${...}` and `$$`."""
    out = bytearray()
    index = {n: i for i, n in enumerate(names) if n}
    while rep:
        i = rep.find(b"$")
        if i < 0:
            break
        out += rep[:i]
        rep = rep[i:]
        if len(rep) > 1 and rep[1] == 0x24:
            out += b"$"
            rep = rep[2:]
            continue
        ref = _find_cap_ref(rep)
        if ref is None:
            out += b"$"
            rep = rep[1:]
            continue
        cap, end = ref
        rep = rep[end:]
        g = cap if isinstance(cap, int) else index.get(cap)
        if g is not None and g < len(groups) and groups[g] is not None:
            out += text[groups[g][0]:groups[g][1]]
    out += rep
    return bytes(out)


class _Split(object):
    """re_bytes.rs:699-721 over the match list of a find_iter."""

    def __init__(self, text, matches):
        self.text, self.ms, self.last = text, iter(matches), 0

    def next(self):
        m = next(self.ms, None)
        if m is None:
            if self.last >= len(self.text):
                return None
            s = self.text[self.last:]
            self.last = len(self.text)
            return s
        s = self.text[self.last:m[0]]
        self.last = m[1]
        return s


class Regex(object):
    """`regex::bytes::Regex` (re_bytes.rs:78-605): Unicode on by default."""

    def __init__(self, pattern, case_insensitive=False, multi_line=False,
                 dot_matches_new_line=False, swap_greed=False, ignore_whitespace=False,
                 unicode=True, size_limit=None, dfa_size_limit=None):
        if isinstance(pattern, str):
            pattern = pattern.encode("utf-8")
        self.pattern = pattern
        flags = _flags(case_insensitive, multi_line, dot_matches_new_line, swap_greed,
                       ignore_whitespace, unicode)
        err = N.rure_error_new()
        opts = _options(size_limit, dfa_size_limit)
        try:
            self._re = N.rure_compile(pattern, len(pattern), flags, opts, err)
            if not self._re:
                raise Error(N.rure_error_message(err).decode("utf-8", "replace"))
        finally:
            N.rure_error_free(err)
            if opts:
                N.rure_options_free(opts)

    def __del__(self):
        re_ = getattr(self, "_re", None)
        if re_ and N is not None and getattr(N, "rure_free", None):
            N.rure_free(re_)
            self._re = None

    # ------------------------------------------------ single haystack (rure_*)
    def is_match(self, text, start=0):
        return bool(N.rure_is_match(self._re, text, len(text), start))

    def find(self, text, start=0):
        m = N.RureMatch()
        if N.rure_find(self._re, text, len(text), start, ctypes.byref(m)):
            return (m.start, m.end)
        return None

    def shortest_match(self, text, start=0):
        e = N.c_size()
        if N.rure_shortest_match(self._re, text, len(text), start, ctypes.byref(e)):
            return e.value
        return None

    def find_iter(self, text):
        """bytes::Regex::find_iter (re_trait.rs:197-221): one batched launch
        over the staged haystack."""
        import torch
        text = bytes(text)
        dev = torch.device("cuda", torch.cuda.current_device())
        buf = torch.frombuffer(bytearray(text) + bytearray(16), dtype=torch.uint8).to(dev)
        _, m = self.find_iter_batch(buf, stride=len(text), length=len(text), count=1)
        return [(int(a), int(b)) for a, b in m.cpu().tolist()]

    def iter_rure(self, text):
        """The C API's iteration (rure_iter_next, regex-capi/src/rure.rs:322-360:
        after an empty match the next search starts one past the previous
        search start, which can revisit positions find_iter skips)."""
        it = N.rure_iter_new(self._re)
        out = []
        try:
            m = N.RureMatch()
            while N.rure_iter_next(it, text, len(text), ctypes.byref(m)):
                out.append((m.start, m.end))
        finally:
            N.rure_iter_free(it)
        return out

    def captures(self, text, start=0):
        """Leftmost-first match with its groups (bytes::Regex::captures,
        re_bytes.rs:227-240): a list of (start, end) | None per group (group 0
        = the whole match), or None without a match."""
        caps = N.rure_captures_new(self._re)
        try:
            if not N.rure_find_captures(self._re, text, len(text), start, caps):
                return None
            return _read_caps(caps)
        finally:
            N.rure_captures_free(caps)

    def captures_iter(self, text):
        """bytes::Regex::captures_iter (CaptureMatches, re_trait.rs:243-273)."""
        out, last_end, last_match = [], 0, None
        while last_end <= len(text):
            g = self.captures(text, last_end)
            if g is None:
                break
            s, e = g[0]
            if s == e:
                last_end = e + 1
                if last_match == e:
                    continue
            else:
                last_end = e
            last_match = e
            out.append(g)
        return out

    def captures_iter_rure(self, text):
        """Successive captures as rure_iter_next_captures iterates them."""
        it = N.rure_iter_new(self._re)
        caps = N.rure_captures_new(self._re)
        out = []
        try:
            while N.rure_iter_next_captures(it, text, len(text), caps):
                out.append(_read_caps(caps))
        finally:
            N.rure_captures_free(caps)
            N.rure_iter_free(it)
        return out

    def captures_len(self):
        return int(N.rure_amd_captures_len(self._re))

    def capture_names(self):
        """Group names in index order, None for unnamed groups (re_bytes.rs:580-590)."""
        it = N.rure_iter_capture_names_new(self._re)
        out = []
        try:
            p = ctypes.c_char_p()
            while N.rure_iter_capture_names_next(it, ctypes.byref(p)):
                out.append(p.value.decode("utf-8") or None)
        finally:
            N.rure_iter_capture_names_free(it)
        return out

    def capture_name_index(self, name):
        i = N.rure_capture_name_index(self._re, name.encode("utf-8"))
        return None if i < 0 else i

    # ------------------------------------ replace / split (re_bytes.rs:316-535)
    def replacen(self, text, limit, rep):
        """Replaces the first `limit` matches (0 = all).  `rep` is bytes with
        `$` expansion, a NoExpand, or a function f(groups, text) -> bytes (the
        reference's FnMut(&Captures) replacer)."""
        text = bytes(text)
        if isinstance(rep, NoExpand) or (isinstance(rep, (bytes, bytearray)) and b"$" not in rep):
            lit = rep.rep if isinstance(rep, NoExpand) else bytes(rep)
            ms = self.find_iter(text)
            if limit:
                ms = ms[:limit]
            out, last = bytearray(), 0
            for s, e in ms:
                out += text[last:s]
                out += lit
                last = e
            return bytes(out + text[last:])
        caps = self.captures_iter(text)
        if limit:
            caps = caps[:limit]
        names = self.capture_names() if not callable(rep) else None
        out, last = bytearray(), 0
        for g in caps:
            s, e = g[0]
            out += text[last:s]
            out += rep(g, text) if callable(rep) else expand(g, names, bytes(rep), text)
            last = e
        return bytes(out + text[last:])

    def replace(self, text, rep):
        return self.replacen(text, 1, rep)

    def replace_all(self, text, rep):
        return self.replacen(text, 0, rep)

    def split(self, text):
        """Fields between matches (re_bytes.rs:699-721)."""
        text = bytes(text)
        sp = _Split(text, self.find_iter(text))
        out = []
        while True:
            x = sp.next()
            if x is None:
                return out
            out.append(x)

    def splitn(self, text, limit):
        """At most `limit` fields, the last being the rest (re_bytes.rs:729-749)."""
        text = bytes(text)
        sp = _Split(text, self.find_iter(text))
        out, n = [], limit
        while n:
            n -= 1
            if n == 0:
                out.append(text[sp.last:])
                break
            x = sp.next()
            if x is None:
                break
            out.append(x)
        return out

    # -------------------------------------------- batches (device tensors)
    def replace_batch(self, haystack, rep, limit=0, offsets=None, stride=None, length=None, count=None,
                      stream=None):
        """replacen over every haystack with a literal replacement (`$` is
        not expanded; NoExpand semantics).  Returns (out, out_offsets): the
        concatenated outputs (uint8) and n+1 int64 offsets into them."""
        import torch
        if isinstance(rep, NoExpand):
            rep = rep.rep
        rep = bytes(rep)
        b = _batch(haystack, offsets, stride, length, count, 0)
        dev = haystack.device
        ooff = torch.empty((b.count + 1,), dtype=torch.int64, device=dev)
        total = torch.zeros((1,), dtype=torch.int64, device=dev)
        cap = haystack.numel() + 1024
        while True:
            out = torch.empty((max(cap, 16) + 16,), dtype=torch.uint8, device=dev)
            _check(N.rure_amd_replace_batch(self._re, ctypes.byref(b), rep, len(rep), limit,
                                            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ooff.data_ptr()), cap,
                                            ctypes.c_void_p(total.data_ptr()), _stream_ptr(stream)), "replace_batch")
            (stream or torch.cuda.current_stream()).synchronize()
            t = int(total.item())
            if t <= cap:
                return out[:t], ooff
            cap = t

    def split_batch(self, haystack, limit=None, offsets=None, stride=None, length=None, count=None,
                    capacity=None, stream=None):
        """split (limit None) / splitn over every haystack.  Returns (counts,
        pieces): fields per haystack and (total, 2) int64 (start, end)."""
        import torch
        b = _batch(haystack, offsets, stride, length, count, 0)
        dev = haystack.device
        lim = (1 << 64) - 1 if limit is None else limit
        counts = torch.empty((b.count,), dtype=torch.int64, device=dev)
        total = torch.zeros((1,), dtype=torch.int64, device=dev)
        cap = capacity if capacity is not None else max(1024, 4 * b.count)
        while True:
            out = torch.empty((max(cap, 1), 2), dtype=torch.int64, device=dev)
            _check(N.rure_amd_split_batch(self._re, ctypes.byref(b), lim, ctypes.c_void_p(counts.data_ptr()),
                                          ctypes.c_void_p(out.data_ptr()), cap, ctypes.c_void_p(total.data_ptr()),
                                          _stream_ptr(stream)), "split_batch")
            (stream or torch.cuda.current_stream()).synchronize()
            t = int(total.item())
            if t <= cap or capacity is not None:
                return counts, out[:min(t, cap)]
            cap = t

    def captures_batch(self, haystack, offsets=None, stride=None, length=None, count=None,
                       start=0, out=None, stream=None):
        """Captures per haystack: an (n, groups, 2) int64 tensor of
        (start, end), -1 where a group did not participate or there is no match."""
        import torch
        b = _batch(haystack, offsets, stride, length, count, start)
        if out is None:
            out = torch.empty((b.count, self.captures_len(), 2), dtype=torch.int64, device=haystack.device)
        _check(N.rure_amd_captures_batch(self._re, ctypes.byref(b), ctypes.c_void_p(out.data_ptr()),
                                         _stream_ptr(stream)), "captures_batch")
        return out

    def find_batch(self, haystack, offsets=None, stride=None, length=None, count=None,
                   start=0, out=None, stream=None):
        """Leftmost-first match per haystack.  Returns an (n, 2) int64 tensor of
        (start, end); -1 (== SIZE_MAX) marks no match."""
        import torch
        b = _batch(haystack, offsets, stride, length, count, start)
        if out is None:
            out = torch.empty((b.count, 2), dtype=torch.int64, device=haystack.device)
        _check(N.rure_amd_find_batch(self._re, ctypes.byref(b), ctypes.c_void_p(out.data_ptr()),
                                     _stream_ptr(stream)), "find_batch")
        return out

    def is_match_batch(self, haystack, offsets=None, stride=None, length=None, count=None,
                       start=0, out=None, stream=None):
        import torch
        b = _batch(haystack, offsets, stride, length, count, start)
        if out is None:
            out = torch.empty((b.count,), dtype=torch.uint8, device=haystack.device)
        _check(N.rure_amd_is_match_batch(self._re, ctypes.byref(b), ctypes.c_void_p(out.data_ptr()),
                                         _stream_ptr(stream)), "is_match_batch")
        return out

    def shortest_match_batch(self, haystack, offsets=None, stride=None, length=None, count=None,
                             start=0, out=None, stream=None):
        import torch
        b = _batch(haystack, offsets, stride, length, count, start)
        if out is None:
            out = torch.empty((b.count,), dtype=torch.int64, device=haystack.device)
        _check(N.rure_amd_shortest_match_batch(self._re, ctypes.byref(b), ctypes.c_void_p(out.data_ptr()),
                                               _stream_ptr(stream)), "shortest_match_batch")
        return out

    def find_iter_batch(self, haystack, offsets=None, stride=None, length=None, count=None, start=0,
                        capacity=None, stream=None):
        """All successive non-overlapping matches of every haystack
        (bytes::Regex::find_iter, re_trait.rs:197-221).  Returns (counts, matches):
        counts = (n,) int64 per haystack, matches = (total, 2) int64 (start, end)
        concatenated in haystack order."""
        import torch
        b = _batch(haystack, offsets, stride, length, count, start)
        dev = haystack.device
        counts = torch.empty((b.count,), dtype=torch.int64, device=dev)
        total = torch.zeros((1,), dtype=torch.int64, device=dev)
        cap = capacity if capacity is not None else max(1024, b.count * 4)
        while True:
            out = torch.empty((max(cap, 1), 2), dtype=torch.int64, device=dev)
            _check(N.rure_amd_find_iter_batch(self._re, ctypes.byref(b), ctypes.c_void_p(counts.data_ptr()),
                                              ctypes.c_void_p(out.data_ptr()), cap,
                                              ctypes.c_void_p(total.data_ptr()), _stream_ptr(stream)),
                   "find_iter_batch")
            (stream or torch.cuda.current_stream()).synchronize()
            t = int(total.item())
            if t <= cap or capacity is not None:
                return counts, out[: min(t, cap)]
            cap = t

    def find_iter_span(self, haystack, lo, hi, length=None, entry=None, capacity=None, stream=None):
        """find_iter restricted to the matches starting in [lo, hi) of one long
        haystack (rure_amd_find_iter_span; sharded / streamed iteration).
        entry: None (fresh start at lo) or the (3,) int64 device tensor a
        previous span returned as its exit.  Returns (count, matches, exit):
        count = (1,) int64, matches = (k, 2) int64, exit = (3,) int64
        (next, last match or -1, fresh)."""
        import torch
        dev = haystack.device
        n = haystack.numel() if length is None else length
        count = torch.zeros((1,), dtype=torch.int64, device=dev)
        exit_ = torch.empty((3,), dtype=torch.int64, device=dev)
        cap = capacity if capacity is not None else max(1024, (hi - lo) // 64)
        ent = ctypes.c_void_p(entry.data_ptr()) if entry is not None else None
        while True:
            out = torch.empty((max(cap, 1), 2), dtype=torch.int64, device=dev)
            _check(N.rure_amd_find_iter_span(self._re, ctypes.c_void_p(haystack.data_ptr()), n, lo, hi, ent,
                                             ctypes.c_void_p(count.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                             cap, ctypes.c_void_p(exit_.data_ptr()), _stream_ptr(stream)),
                   "find_iter_span")
            (stream or torch.cuda.current_stream()).synchronize()
            t = int(count.item())
            if t <= cap or capacity is not None:
                return count, out[: min(t, cap)], exit_
            cap = t

    # ----------------------------------------------------------- diagnostics
    def match_info(self):
        """The reference's engine choice for this regex (exec.rs:1130-1210)
        and the literal searchers it rests on."""
        i = N.MatchInfo()
        _check(N.rure_amd_match_info_get(self._re, ctypes.byref(i)), "match_info")
        return {"match_type": MATCH_TYPES[i.match_type], "prefix_matcher": i.prefix_matcher,
                "suffix_matcher": i.suffix_matcher, "prefix_len": i.prefix_len, "suffix_len": i.suffix_len,
                "prefix_complete": bool(i.prefix_complete), "suffix_complete": bool(i.suffix_complete),
                "lcp_chars": i.lcp_chars, "lcs_chars": i.lcs_chars, "lcs": bytes(i.lcs[:i.lcs_bytes])}

    def exec_literals(self, which="prefixes"):
        """The unambiguous prefix / suffix literal set the reference builds (exec.rs:308-321)."""
        return _de_lits(_call_out(N.rure_amd_exec_literals_export, self._re, 0 if which == "prefixes" else 1))

    def dfa_info(self, which=0):
        info = N.DfaInfo()
        rc = N.rure_amd_dfa_info_get(self._re, which, ctypes.byref(info))
        return {k: getattr(info, k) for k, _ in N.DfaInfo._fields_} if rc == N.OK else None

    def first_bytes(self):
        """The first-byte start rule of the chunked find_iter (bytes of F, or
        None when the rule does not hold)."""
        buf = (ctypes.c_uint8 * 4)()
        n = N.rure_amd_first_byte_export(self._re, buf)
        return bytes(buf[:n]) if n > 0 else None

    def lex_table(self, ascii=False):
        """The find_iter lexer table: (flat uint8 table: the entry after byte
        b from entry e is table[76 e + b], start entry), or None (see
        rure_amd.h rure_amd_lex_export).  ascii=True: the ASCII shadow's
        (rure_amd_lex_ascii_export)."""
        import numpy as np
        if ascii:
            ex = lambda t, n, s: N.rure_amd_lex_ascii_export(self._re, 0, t, n, s)  # noqa: E731
        else:
            ex = lambda t, n, s: N.rure_amd_lex_export(self._re, t, n, s)  # noqa: E731
        n = ex(None, 0, None)
        if n <= 0:
            return None
        t = np.zeros(n, dtype=np.uint8)
        s0 = ctypes.c_uint32()
        ex(t.ctypes.data, n, ctypes.byref(s0))
        return t, s0.value

    def run_class(self, ascii=False):
        """The find_iter run engine's class (rure_amd_run_class_export): a
        256-entry uint8 array (bit 0: the byte is in C, bit 1: it quits) if
        the regex is C+ (on ASCII text when ascii=True), else None."""
        import numpy as np
        c = np.zeros(256, dtype=np.uint8)
        return c if N.rure_amd_run_class_export(self._re, 1 if ascii else 0, c.ctypes.data) == 1 else None

    def run_code_points(self):
        """The run engine's code point bitmap for a Unicode class C+
        (rure_amd_run_cp_export): a uint32 array of 0x110000 bits, or None
        when the engine reads no UTF-8 for this regex."""
        import numpy as np
        n = N.rure_amd_run_cp_export(self._re, None, 0)
        if n <= 0:
            return None
        b = np.zeros(n, dtype=np.uint32)
        N.rure_amd_run_cp_export(self._re, b.ctypes.data, n)
        return b

    def lex4_table(self, ascii=False):
        """The four-bytes-per-step lexer table (rure_amd_lex4_export): (flat
        uint8 table, start row), or None.  ascii=True: the ASCII shadow's."""
        import numpy as np
        if ascii:
            ex = lambda t, n, s: N.rure_amd_lex_ascii_export(self._re, 1, t, n, s)  # noqa: E731
        else:
            ex = lambda t, n, s: N.rure_amd_lex4_export(self._re, t, n, s)  # noqa: E731
        n = ex(None, 0, None)
        if n <= 0:
            return None
        t = np.zeros(n, dtype=np.uint8)
        s0 = ctypes.c_uint32()
        ex(t.ctypes.data, n, ctypes.byref(s0))
        return t, s0.value

    def program(self, which):
        """Compiled byte program (0 fwd DFA, 1 reverse DFA, 2 NFA): (info, insts)."""
        return _export(N.rure_amd_program_export, self._re, which)

    def uses_dfa(self):
        """True if batched searches run the DFA kernels (else the Pike VM kernel)."""
        return N.rure_amd_uses_dfa(self._re) == 1

    def shiftand(self):
        """The Shift-And image the find_iter string-set engine runs
        (iter_spec_sa_kernel), or None: (bits, masks (256 u64), init, final,
        string length)."""
        import numpy as np
        mask = np.zeros(256, dtype=np.uint64)
        init, fin, ln = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint32(0)
        bits = N.rure_amd_shiftand_export(self._re, mask.ctypes.data, ctypes.byref(init), ctypes.byref(fin),
                                          ctypes.byref(ln))
        if bits <= 0:
            return None
        return int(bits), [int(x) for x in mask], init.value, fin.value, ln.value

    def literals(self):
        """The regex as a finite string set in leftmost-first priority order, as
        the literal find_iter engine uses it, or None if it is not one."""
        import numpy as np
        n = N.rure_amd_literals_export(self._re, None, None, 0)
        if n <= 0:
            return None
        lens = np.zeros(n, dtype=np.uint32)
        buf = np.zeros(32 * n, dtype=np.uint8)
        N.rure_amd_literals_export(self._re, lens.ctypes.data, buf.ctypes.data, n)
        return [bytes(buf[32 * i:32 * i + int(lens[i])]) for i in range(n)]

    def nfa_tables(self):
        """Pike VM closure tables of the NFA kernel: (info, leaves, cl_off, entries)."""
        return _nfa_export(N.rure_amd_nfa_export, self._re)

    def nfa_saves(self):
        """Capture slots set by each closure entry: (save_off, save_slot)."""
        import numpy as np
        n = N.c_size()
        _check(N.rure_amd_nfa_saves_export(self._re, None, None, ctypes.byref(n)), "nfa_saves_export")
        ents = self.nfa_tables()[0]["entries"]
        off = np.zeros(ents + 1, dtype=np.uint32)
        slot = np.zeros(max(n.value, 1), dtype=np.uint16)
        _check(N.rure_amd_nfa_saves_export(self._re, off.ctypes.data, slot.ctypes.data, ctypes.byref(n)),
               "nfa_saves_export")
        return off, slot[: n.value]

    def dfa_tables(self, which=0):
        import numpy as np
        info = self.dfa_info(which)
        if info is None:
            return None
        n = info["states"]
        trans = np.zeros(n * 256, dtype=np.uint32)
        eof = np.zeros(n, dtype=np.uint8)
        start = np.zeros(128, dtype=np.uint32)
        _check(N.rure_amd_dfa_export(self._re, which, trans.ctypes.data, eof.ctypes.data, start.ctypes.data),
               "dfa_export")
        if which == 2:
            strip = np.zeros(n, dtype=np.uint32)
            _check(N.rure_amd_dfa_strip_export(self._re, strip.ctypes.data), "dfa_strip_export")
            info["strip"] = strip
        return info, trans.reshape(n, 256), eof, start


def replace_all_chain(regexes, reps, haystack, length=None, capacity=None, stream=None):
    """replace_all of each regex in turn over one haystack, every step on the
    previous step's output (rure_amd_replace_all_chain: regexes whose matches
    are single bytes of one class, replacements of 1-64 bytes, e.g. the
    regex-dna IUB substitutions).  Only enqueues.  Returns (out, lengths):
    the final text in out[:lengths[-1]] (a device tensor of capacity + 16
    bytes) and the n + 1 lengths (device int64).  If lengths[-1] exceeds
    capacity the output was cut: call again with capacity >= lengths[-1]."""
    import torch
    n = len(regexes)
    length = haystack.numel() - 16 if length is None else length
    capacity = length + length // 2 + 4096 if capacity is None else capacity
    dev = haystack.device
    bufs = [torch.empty((capacity + 16,), dtype=torch.uint8, device=dev) for _ in range(min(n, 2) or 1)]
    for b in bufs:
        b[capacity:].zero_()
    lengths = torch.empty((n + 1,), dtype=torch.int64, device=dev)
    reps = [bytes(r.rep if isinstance(r, NoExpand) else r) for r in reps]
    res_arr = (ctypes.c_void_p * max(n, 1))(*[r._re for r in regexes])
    rep_bufs = [ctypes.create_string_buffer(r, max(len(r), 1)) for r in reps]
    rep_arr = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(b) for b in rep_bufs])
    len_arr = (ctypes.c_size_t * max(n, 1))(*[len(r) for r in reps])
    _check(N.rure_amd_replace_all_chain(res_arr, rep_arr, len_arr, n, ctypes.c_void_p(haystack.data_ptr()), length,
                                        ctypes.c_void_p(bufs[0].data_ptr()),
                                        ctypes.c_void_p(bufs[-1].data_ptr()), capacity,
                                        ctypes.c_void_p(lengths.data_ptr()), _stream_ptr(stream)),
           "replace_all_chain")
    out = haystack if n == 0 else bufs[0] if n % 2 else bufs[1]
    return out, lengths


def find_iter_span_multi(regexes, haystack, lo, hi, length=None, entries=None, capacities=None, stream=None):
    """Regex.find_iter_span for several regexes over the same span [lo, hi)
    (rure_amd_find_iter_span_multi: finite string sets of one common length,
    e.g. the regex-dna variants, are scanned in one pass over the text).
    entries: None or a list of (3,) device exits (None items: fresh starts).
    Returns [(count, matches, exit), ...] in the order of `regexes`, each
    exactly what that regex's find_iter_span returns.  With capacities given
    the outputs are not resized (a count above its capacity: truncated)."""
    import torch
    k = len(regexes)
    dev = haystack.device
    n = haystack.numel() if length is None else length
    caps = list(capacities) if capacities is not None else [max(1024, (hi - lo) // 64)] * k
    counts = [torch.zeros((1,), dtype=torch.int64, device=dev) for _ in range(k)]
    exits = [torch.empty((3,), dtype=torch.int64, device=dev) for _ in range(k)]
    VP = ctypes.c_void_p
    res = (VP * k)(*[r._re for r in regexes])
    ent = None
    if entries is not None:
        ent = (VP * k)(*[VP(e.data_ptr()) if e is not None else None for e in entries])
    while True:
        outs = [torch.empty((max(c, 1), 2), dtype=torch.int64, device=dev) for c in caps]
        _check(N.rure_amd_find_iter_span_multi(res, k, VP(haystack.data_ptr()), n, lo, hi, ent,
                                               (VP * k)(*[VP(c.data_ptr()) for c in counts]),
                                               (VP * k)(*[VP(o.data_ptr()) for o in outs]),
                                               (ctypes.c_size_t * k)(*caps),
                                               (VP * k)(*[VP(x.data_ptr()) for x in exits]), _stream_ptr(stream)),
               "find_iter_span_multi")
        if capacities is not None:
            return [(counts[i], outs[i], exits[i]) for i in range(k)]
        (stream or torch.cuda.current_stream()).synchronize()
        tot = [int(c.item()) for c in counts]
        if all(t <= c for t, c in zip(tot, caps)):
            return [(counts[i], outs[i][: tot[i]], exits[i]) for i in range(k)]
        caps = [max(t, c) for t, c in zip(tot, caps)]


def _read_caps(caps):
    out = []
    m = N.RureMatch()
    for i in range(N.rure_captures_len(caps)):
        out.append((m.start, m.end) if N.rure_captures_at(caps, i, ctypes.byref(m)) else None)
    return out


def _nfa_export(fn, handle):
    import numpy as np
    info = N.NfaInfo()
    _check(fn(handle, ctypes.byref(info), None, None, None), "nfa_export")
    leaves = np.zeros(max(info.leaves, 1) * 3, dtype=np.uint32)
    cl_off = np.zeros(info.closures + 1, dtype=np.uint32)
    ent = np.zeros(max(info.entries, 1) * 2, dtype=np.uint32)
    _check(fn(handle, ctypes.byref(info), leaves.ctypes.data, cl_off.ctypes.data, ent.ctypes.data), "nfa_export")
    d = {k: getattr(info, k) for k, _ in N.NfaInfo._fields_}
    return d, leaves[: info.leaves * 3].reshape(-1, 3), cl_off, ent[: info.entries * 2].reshape(-1, 2)


def _export(fn, handle, which):
    import numpy as np
    info = N.ProgInfo()
    n = fn(handle, which, ctypes.byref(info), None, 0)
    if n < 0:
        raise ValueError("no such program")
    arr = np.zeros(max(n, 1) * 12, dtype=np.uint8)
    fn(handle, which, ctypes.byref(info), arr.ctypes.data, n)
    return info, arr[: n * 12]


class RegexSet(object):
    """`regex::bytes::RegexSet` (re_set.rs:86-254)."""

    def __init__(self, patterns, case_insensitive=False, multi_line=False,
                 dot_matches_new_line=False, swap_greed=False, ignore_whitespace=False,
                 unicode=True, size_limit=None, dfa_size_limit=None):
        pats = [p.encode("utf-8") if isinstance(p, str) else p for p in patterns]
        self.patterns = pats
        arr = (ctypes.c_char_p * max(len(pats), 1))(*pats)
        lens = (N.c_size * max(len(pats), 1))(*[len(p) for p in pats])
        flags = _flags(case_insensitive, multi_line, dot_matches_new_line, swap_greed,
                       ignore_whitespace, unicode)
        err = N.rure_error_new()
        opts = _options(size_limit, dfa_size_limit)
        try:
            self._set = N.rure_compile_set(arr, lens, len(pats), flags, opts, err)
            if not self._set:
                raise Error(N.rure_error_message(err).decode("utf-8", "replace"))
        finally:
            N.rure_error_free(err)
            if opts:
                N.rure_options_free(opts)

    def __del__(self):
        s = getattr(self, "_set", None)
        if s and N is not None and getattr(N, "rure_set_free", None):
            N.rure_set_free(s)
            self._set = None

    def __len__(self):
        return N.rure_set_len(self._set)

    def is_match(self, text, start=0):
        return bool(N.rure_set_is_match(self._set, text, len(text), start))

    def matches(self, text, start=0):
        n = len(self)
        buf = (ctypes.c_bool * max(n, 1))()
        N.rure_set_matches(self._set, text, len(text), start, buf)
        return [i for i in range(n) if buf[i]]

    @property
    def words(self):
        """u64 mask words per haystack in matches_batch's output."""
        return max(1, (len(self) + 63) // 64)

    def matches_batch(self, haystack, offsets=None, stride=None, length=None, count=None,
                      start=0, out=None, stream=None):
        """Bit masks of the patterns matching each haystack: an (n,) int64
        tensor (bit j <=> pattern j matched) for sets of up to 64 patterns,
        else (n, words) with pattern j at bit j % 64 of word j // 64."""
        import torch
        b = _batch(haystack, offsets, stride, length, count, start)
        w = self.words
        if out is None:
            shape = (b.count,) if len(self) <= 64 else (b.count, w)
            out = torch.empty(shape, dtype=torch.int64, device=haystack.device)
        elif (out.dtype != torch.int64 or not out.is_contiguous() or not out.is_cuda
              or out.numel() < b.count * w):
            # the kernels write count * words int64 words: anything smaller
            # (e.g. an (n,) tensor for a set of more than 64 patterns) would
            # be written out of bounds
            raise ValueError("out must be a contiguous int64 CUDA tensor of at least %d x %d words"
                             % (b.count, w))
        _check(N.rure_amd_set_matches_batch_words(self._set, ctypes.byref(b), ctypes.c_void_p(out.data_ptr()), w,
                                                  _stream_ptr(stream)), "matches_batch")
        return out

    def program(self, which):
        return _export(N.rure_amd_set_program_export, self._set, which)

    def uses_dfa(self):
        return N.rure_amd_set_uses_dfa(self._set) == 1

    def core_tables(self):
        """Core form of a large set's DFA (None if the set uses the byte-row
        kernel): (info, class map, hot table, gcore, gout, eof, start,
        code masks)."""
        import numpy as np
        info = N.CoreInfo()
        if N.rure_amd_set_core_export(self._set, ctypes.byref(info), None, None, None, None, None) != N.OK:
            return None
        d = {k: getattr(info, k) for k, _ in N.CoreInfo._fields_}
        lds = np.zeros(info.lds_bytes, dtype=np.uint8)
        gcore = np.zeros(info.ncores * info.K, dtype=np.uint16)
        gout = np.zeros(info.ncores * info.K, dtype=np.uint64)
        eof = np.zeros(info.ncores, dtype=np.uint64)
        start = np.zeros(128, dtype=np.uint16)
        _check(N.rure_amd_set_core_export(self._set, ctypes.byref(info), lds.ctypes.data, gcore.ctypes.data,
                                          gout.ctypes.data, eof.ctypes.data, start.ctypes.data), "set_core_export")
        K, hot = info.K, info.hot
        # rows of K + 1 entries: column K is the identity (the class of the
        # bytes outside a masked head / tail chunk); then the 64 code masks
        t_end = 256 + (hot + 1) * (K + 1) * 2
        hot_tab = lds[256:t_end].view(np.uint16).reshape(hot + 1, K + 1)
        mt = (t_end + 7) & ~7
        masktab = lds[mt:mt + 512].view(np.uint64).copy()
        return d, lds[:256].copy(), hot_tab, gcore.reshape(-1, K), gout.reshape(-1, K), eof, start, masktab

    def dfa_tables(self):
        """Set DFA: (info, trans (states, 256), eof_mask, now_mask, start)."""
        import numpy as np
        info = self.dfa_info()
        if info is None or not info.get("ok"):
            return None
        n = info["states"]
        trans = np.zeros(n * 256, dtype=np.uint32)
        eof = np.zeros(n, dtype=np.uint64)
        now = np.zeros(n, dtype=np.uint64)
        start = np.zeros(128, dtype=np.uint32)
        _check(N.rure_amd_set_dfa_export(self._set, trans.ctypes.data, eof.ctypes.data, now.ctypes.data,
                                         start.ctypes.data), "set_dfa_export")
        return info, trans.reshape(n, 256), eof, now, start

    def nfa_tables(self):
        return _nfa_export(N.rure_amd_set_nfa_export, self._set)

    def dfa_info(self):
        info = N.DfaInfo()
        rc = N.rure_amd_set_dfa_info_get(self._set, ctypes.byref(info))
        return {k: getattr(info, k) for k, _ in N.DfaInfo._fields_} if rc == N.OK else None
