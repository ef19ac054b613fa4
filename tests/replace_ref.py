"""TEST INFRASTRUCTURE: bytes::Regex::replacen / split / splitn restated over
the oracle (re_bytes.rs:489-535, 699-749; CaptureMatches re_trait.rs:243-273),
the checker for the GPU replace / split paths.  `$` expansion uses
regex_amd.expand, which tests/test_replace_host.py and the reference's
expand! vectors pin."""
import regex_amd as R


def captures_iter(o, text):
    out, last_end, last_match = [], 0, None
    while last_end <= len(text):
        c = o.captures(text, last_end)
        if c is None:
            break
        s, e = c[0]
        if s == e:
            last_end = e + 1
            if last_match == e:
                continue
        else:
            last_end = e
        last_match = e
        out.append(c)
    return out


def replacen(o, names, text, limit, rep, literal):
    if literal or b"$" not in rep:
        ms = o.find_iter(text)
        if limit:
            ms = ms[:limit]
        out, last = bytearray(), 0
        for s, e in ms:
            out += text[last:s] + rep
            last = e
        return bytes(out + text[last:])
    caps = captures_iter(o, text)
    if limit:
        caps = caps[:limit]
    out, last = bytearray(), 0
    for g in caps:
        out += text[last:g[0][0]] + R.expand(g, names, rep, text)
        last = g[0][1]
    return bytes(out + text[last:])


class _Split(object):
    def __init__(self, text, ms):
        self.text, self.ms, self.last = text, iter(ms), 0

    def next(self):
        m = next(self.ms, None)
        if m is None:
            if self.last >= len(self.text):
                return None
            s, self.last = self.text[self.last:], len(self.text)
            return s
        s, self.last = self.text[self.last:m[0]], m[1]
        return s


def split(o, text):
    sp, out = _Split(text, o.find_iter(text)), []
    while True:
        x = sp.next()
        if x is None:
            return out
        out.append(x)


def splitn(o, text, n):
    sp, out = _Split(text, o.find_iter(text)), []
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
