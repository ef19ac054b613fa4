#!/usr/bin/env python3
r"""Unicode parity fixtures that do not go through the product's front end.

The oracle runs the programs the product's own parser and Unicode tables
compile, so a wrong class (a parser slip, a table error) would make the GPU
and the oracle agree on the wrong answer.  These fixtures come from Python's
stdlib `re` in `str` mode over valid UTF-8 text instead, converted to byte
offsets, for the patterns whose classes are Unicode:

    \w+  \pL+  \S+  \d+  .+  (?i)[a-zé]+  \d{4}-\d{2}-\d{2}  \w+@\w+\.\w+

Python's Unicode version (and its definitions of \w and \s) differ from the
reference's Unicode 10 perl classes, so the text is drawn only from code
points on which the two agree for every class involved.  The reference side
of that check reads the reference's tables as data, from
regex-syntax/src/unicode.rs: PERLW (:4725), PERLD = Nd_table (:4721, :1821),
PERLS = White_Space_table (:4723, :4548), L_table (:540) and the simple case
folding pairs C_plus_S_both_table (:4995, applied as lib.rs:871-890 does).
Python stands in for the engine: \pL+ is written [^\W\d_]+ (letters, once
the pool agrees), `.` is the same "anything but \n" in both.

Writes tests/golden/unicode_re_fixtures.json.gz (inputs + expected byte
spans: data only).  Run in the build container, where /root/reference is:
    python tests/golden/gen_unicode_fixtures.py
"""
import gzip
import json
import os
import random
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
UNICODE_RS = "/root/reference/regex-syntax/src/unicode.rs"

# (pattern as the product takes it, the same pattern for Python's re)
PATTERNS = [
    (r"\w+", r"\w+"),
    (r"\pL+", r"[^\W\d_]+"),
    (r"\S+", r"\S+"),
    (r"\d+", r"\d+"),
    (r".+", r".+"),
    (r"(?i)[a-zé]+", r"(?i)[a-zé]+"),
    (r"\d{4}-\d{2}-\d{2}", r"\d{4}-\d{2}-\d{2}"),
    (r"\w+@\w+\.\w+", r"\w+@\w+\.\w+"),
]

# candidate code points: ASCII, Latin-1/Extended, Greek, Cyrillic, Arabic and
# Devanagari letters and digits, fullwidth digits, CJK, Hangul, spaces other
# than ASCII, marks, symbols, astral letters and symbols (1-4 byte encodings)
CANDIDATES = (
    [chr(c) for c in range(0x20, 0x7F)] + ["\n", "\t"] +
    list("éÉüÜñÑßàÀçÇøØæÆµªº²³½¡¿«»·×÷§¶°±") +
    list("ĀāĂăĄąĆćČčĎďĐđĒēĘęĚěĞğĦħĲĳĿŀŁłŃńŇňŐőŒœŘřŚśŠšŢţŤťŮůŰűŸŹźŻżŽžƒǅǆ") +
    list("ΑαΒβΓγΔδΩωάέήίόύώΐϊϋ") + list("АаБбВвГгДдЖжЯяЁёЩщЪъЬь") +
    list("ابتثجحخدذرزسشصضطظعغفقكلمنهوي") + [chr(c) for c in range(0x660, 0x66A)] +
    [chr(c) for c in range(0x6F0, 0x6FA)] + list("कखगघङचछजझटठडढणतथदधनपफबभमयरलवशसह") +
    [chr(c) for c in range(0x966, 0x970)] + [chr(c) for c in range(0xE50, 0xE5A)] +
    [chr(c) for c in range(0xFF10, 0xFF1A)] + list("ＡＢＣａｂｃ") +
    list("中文字符日本語漢字한국어あいうえおアイウエオ") +
    [" ", " ", " ", " ", " ", " ", " ", " ", " ", " ", "　",
     "\u0085", "\u001c", "\u001f", "\u000b", "\u000c", "\u000d"] +
    ["́", "̈", "ः", "⃝", "‍", "‌"] +
    list("€£¥₹—–…‘’“”•†‡‰′″←→↑↓∀∂∃∅∈∑√∞≈≠≤≥⌘⌚☃★☆♠♣♥♦✓✗") +
    ["\U0001F600", "\U0001F680", "\U0001F44D", "\U0001D400", "\U0001D538", "\U0001D56B", "\U00010400",
     "\U00010428", "\U0001F130", "\U00020000", "\U0002A6D6", "\U0001E900", "\U0001E922", "\U0001D7CE",
     "\U000104A0", "\U00011066"] +
    ["K", "ſ", "İ", "ı", "ẞ", "µ", "μ", "Μ", "ι"]
)


def ref_table(src, name):
    """The ranges of `pub const <name>: &'static [(char, char)]` in unicode.rs."""
    m = re.search(r"pub const %s: &'static \[\(char, char\)\] = &\[(.*?)\];" % re.escape(name), src, re.S)
    assert m, name
    body = m.group(1)
    lit = r"'(\\u\{[0-9a-fA-F]+\}|\\.|[^'\\])'"

    def ch(s):
        if s.startswith("\\u{"):
            return int(s[3:-1], 16)
        if s.startswith("\\"):
            return ord({"n": "\n", "t": "\t", "r": "\r", "'": "'", "\\": "\\", "0": "\0"}[s[1]])
        return ord(s)

    return [(ch(a), ch(b)) for a, b in re.findall(r"\(" + lit + r",\s*" + lit + r"\)", body)]


def member(ranges, c):
    return any(a <= c <= b for a, b in ranges)


def agreeing_pool():
    src = open(UNICODE_RS, encoding="utf-8").read()
    perlw = ref_table(src, "PERLW")
    nd = ref_table(src, "Nd_table")
    ws = ref_table(src, "White_Space_table")
    letters = ref_table(src, "L_table")
    fold = ref_table(src, "C_plus_S_both_table")
    ci_base = set(range(ord("a"), ord("z") + 1)) | {ord("é")}
    ci = set(ci_base) | {b for a, b in fold if a in ci_base}
    py = {k: re.compile(v) for k, v in
          {"w": r"\w", "d": r"\d", "s": r"\s", "L": r"[^\W\d_]", "ci": r"(?i)[a-zé]"}.items()}
    keep, dropped = [], []
    for ch in dict.fromkeys(CANDIDATES):
        c = ord(ch)
        ref = {"w": member(perlw, c), "d": member(nd, c), "s": member(ws, c), "L": member(letters, c),
               "ci": c in ci}
        ok = all(bool(py[k].fullmatch(ch)) == ref[k] for k in ref) and ch.isalpha() == ref["L"]
        (keep if ok else dropped).append(ch)
    return keep, dropped


def text(rng, pool, nchars):
    """Words of pool characters, separators, dates and address-like runs."""
    seps = [c for c in pool if not re.fullmatch(r"\w", c)]
    word = [c for c in pool if re.fullmatch(r"\w", c)]
    digits = [c for c in pool if re.fullmatch(r"\d", c)]
    out, n = [], 0
    while n < nchars:
        k = rng.random()
        if k < 0.08:
            d = rng.choice([digits, [c for c in digits if c.isascii()]])
            t = "".join(rng.choice(d) for _ in range(4)) + "-" + "".join(rng.choice(d) for _ in range(2)) + \
                rng.choice(["-", "–", "/"]) + "".join(rng.choice(d) for _ in range(rng.choice([1, 2, 2, 3])))
        elif k < 0.14:
            t = "".join(rng.choice(word) for _ in range(rng.randint(1, 6))) + "@" + \
                "".join(rng.choice(word) for _ in range(rng.randint(1, 5))) + rng.choice([".", ".", "..", "。"]) + \
                "".join(rng.choice(word) for _ in range(rng.randint(0, 4)))
        elif k < 0.75:
            t = "".join(rng.choice(word) for _ in range(rng.randint(1, 9)))
        else:
            t = "".join(rng.choice(seps) for _ in range(rng.randint(1, 3)))
        out.append(t)
        n += len(t)
    return "".join(out)[:nchars]


def byte_spans(pat, s):
    """finditer spans of `pat` over str s, as UTF-8 byte offsets (flat list)."""
    pre = [0]
    for ch in s:
        pre.append(pre[-1] + len(ch.encode()))
    flat = []
    for m in re.finditer(pat, s):
        assert m.end() > m.start()  # no pattern here matches the empty string
        flat += [pre[m.start()], pre[m.end()]]
    return flat


def fixed(rng, pool, n, L):
    """n haystacks of exactly L bytes (characters appended while they fit,
    then ASCII spaces), as str."""
    out = []
    for _ in range(n):
        s = text(rng, pool, L)
        b = 0
        cut = 0
        for i, ch in enumerate(s):
            w = len(ch.encode())
            if b + w > L:
                break
            b += w
            cut = i + 1
        out.append(s[:cut] + " " * (L - b))
    return out


def main():
    pool, dropped = agreeing_pool()
    assert "\u0301" in dropped and "\u0131" in dropped  # the check bites (a mark, dotless i)
    rng = random.Random(0x0C0DE)
    ragged = [text(rng, pool, rng.choice([0, 1, 2, 7, 15, 16, 17, 63, 64, 65, 200, 1000, 3000]))
              for _ in range(300)]
    long_ = [text(rng, pool, 1 << 15), text(rng, pool, 3 << 14)]
    stride = fixed(rng, pool, 1024, 256)
    fx = {"note": "generated by tests/golden/gen_unicode_fixtures.py with Python's re in str mode over "
                  "code points whose classes agree with the reference's Unicode 10 tables (data only)",
          "python": sys.version.split()[0], "pool": "".join(pool), "dropped": "".join(dropped),
          "patterns": [p for p, _ in PATTERNS], "ragged": ragged, "long": long_, "stride": stride,
          "stride_len": 256, "spans": {}}
    for p, q in PATTERNS:
        fx["spans"][p] = {"ragged": [byte_spans(q, s) for s in ragged],
                          "long": [byte_spans(q, s) for s in long_],
                          "stride": [byte_spans(q, s)[:2] for s in stride]}
    with gzip.open(os.path.join(HERE, "unicode_re_fixtures.json.gz"), "wt", encoding="utf-8") as f:
        json.dump(fx, f, ensure_ascii=False)
    print("pool %d code points, dropped %d: %s" % (len(pool), len(dropped), "".join(dropped).encode("unicode_escape")))


if __name__ == "__main__":
    main()
