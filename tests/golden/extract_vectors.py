#!/usr/bin/env python3
"""Extract the reference's own golden vectors into JSON fixtures.

Reads (as text, in the build container) the declarative test vectors of the
reference `regex` 0.2.5 that its `bytes::Regex` test target runs
(tests/test_default_bytes.rs includes api, bytes, crazy, flags, fowler,
multiline, noparse, regression, replace, set, shortest_match, suffix_reverse,
unicode, word_boundary, word_boundary_ascii, plus its own inline mat!s) and the
bench known answers (bench/src/sherlock.rs, bench/src/regexdna.rs,
examples/regexdna-output.txt), and writes:

  tests/golden/reference_vectors.json   mat!/matiter!/matset!/nomatset!/ismatch!/noparse!,
                                        replace!/expand!/split!
  tests/golden/known_counts.json        find_iter counts on the bench corpora
  tests/golden/sherlock.txt.gz          corpus data (bench/src/data/sherlock.txt)
  tests/golden/regexdna-input.txt.gz    corpus data (examples/regexdna-input.txt)

Only inputs and expected outputs are written (data), never reference code.
"""
import gzip
import json
import os
import re
import sys

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

MODULES = ["api", "bytes", "crazy", "flags", "fowler", "multiline", "noparse", "regression",
           "replace", "set", "shortest_match", "suffix_reverse", "unicode", "word_boundary",
           "word_boundary_ascii"]
MACROS = ("mat", "matiter", "matset", "nomatset", "ismatch", "noparse", "replace", "expand", "split")


class Lit(object):
    def __init__(self, kind, val):
        self.kind, self.val = kind, val  # kind: str | bytes

    def as_bytes(self):
        return self.val.encode("utf-8") if self.kind == "str" else self.val


def parse_string(s, i):
    """Parses a Rust string/byte-string literal starting at s[i]; returns (Lit, next_i)."""
    is_bytes = False
    if s[i] == "b" and s[i + 1] in "\"r":
        is_bytes = True
        i += 1
    if s[i] == "r":
        j = i + 1
        hashes = 0
        while s[j] == "#":
            hashes += 1
            j += 1
        assert s[j] == '"'
        end = s.index('"' + "#" * hashes, j + 1)
        body = s[j + 1:end]
        val = body.encode("latin-1") if is_bytes else body
        return Lit("bytes" if is_bytes else "str", val), end + 1 + hashes
    assert s[i] == '"', s[i:i + 20]
    j = i + 1
    out = []  # list of ints (bytes) or str chars
    while s[j] != '"':
        c = s[j]
        if c == "\\":
            n = s[j + 1]
            if n == "\n":  # line continuation: skip whitespace
                j += 2
                while s[j] in " \t\n\r":
                    j += 1
                continue
            simple = {"n": "\n", "r": "\r", "t": "\t", "\\": "\\", "0": "\0", "'": "'", '"': '"'}
            if n in simple:
                out.append(simple[n])
                j += 2
            elif n == "x":
                v = int(s[j + 2:j + 4], 16)
                out.append(v if is_bytes else chr(v))
                j += 4
            elif n == "u":
                assert s[j + 2] == "{"
                k = s.index("}", j + 3)
                out.append(chr(int(s[j + 3:k].replace("_", ""), 16)))
                j = k + 1
            else:
                raise ValueError("escape \\%s" % n)
        else:
            out.append(c)
            j += 1
    if is_bytes:
        b = bytearray()
        for x in out:
            if isinstance(x, int):
                b.append(x)
            else:
                b.extend(x.encode("utf-8"))
        return Lit("bytes", bytes(b)), j + 1
    return Lit("str", "".join(out)), j + 1


def split_args(s, i):
    """s[i] is just after '(' of a macro call; returns (list of arg strings, index after ')')."""
    args, depth, cur, j = [], 0, [], i
    while True:
        c = s[j]
        if c in "\"" or (c in "rb" and re.match(r'(b?r#*"|b")', s[j:j + 4]) and not s[j - 1].isalnum()
                         and s[j - 1] != "_"):
            lit_start = j
            _, j = parse_string(s, j)
            cur.append(s[lit_start:j])
            continue
        if c == "/" and s[j + 1] == "/":
            j = s.index("\n", j)
            continue
        if c in "([{":
            depth += 1
        elif c in ")]}":
            if depth == 0:
                args.append("".join(cur).strip())
                return [a for a in args if a != ""], j + 1
            depth -= 1
        if c == "," and depth == 0:
            args.append("".join(cur).strip())
            cur = []
            j += 1
            continue
        cur.append(c)
        j += 1


def parse_value(a):
    a = a.strip()
    m = re.match(r"^(t|no_expand)!\((.*)\)$", a, re.S)
    if m:  # tests/macros_bytes.rs:3,8-13: text as bytes; NoExpand(text)
        lit = parse_value(m.group(2))
        return ("literal" if m.group(1) == "no_expand" else "expand", lit)
    if a.startswith("R(") and a.endswith(")"):
        return parse_value(a[2:-1])
    if re.match(r'^(b?r#*"|b?")', a):
        lit, k = parse_string(a, 0)
        if a[k:].strip():
            raise ValueError("trailing: " + a)
        return lit
    if a == "None":
        return None
    m = re.match(r"^Some\(\(\s*(\d+)\s*,\s*(\d+)\s*\)\)$", a)
    if m:
        return (int(m.group(1)), int(m.group(2)))
    m = re.match(r"^\(\s*(\d+)\s*,\s*(\d+)\s*\)$", a)
    if m:
        return (int(m.group(1)), int(m.group(2)))
    if a in ("true", "false"):
        return a == "true"
    if re.match(r"^\d+$", a):
        return int(a)
    if a.startswith("&["):
        inner, _ = split_args(a, 2)
        return [parse_value(x) for x in inner]
    if "let xs: &[&str] = &[]" in a:
        return []
    raise ValueError("unparsed arg: " + a[:60])


def scan_file(path, vectors, skipped):
    s = open(path, encoding="utf-8").read()
    base = os.path.relpath(path, REF)
    for m in re.finditer(r"(?m)^\s*(%s)!\(" % "|".join(MACROS), s):
        kind = m.group(1)
        line = s.count("\n", 0, m.start()) + 1
        try:
            raw, _ = split_args(s, m.end())
            name = raw[0]
            vals = [parse_value(x) for x in raw[(2 if kind == "replace" else 1):]]
        except Exception as e:  # noqa
            skipped.append("%s:%d %s (%s)" % (base, line, kind, e))
            continue
        src = "%s:%d" % (base, line)
        if kind == "mat":
            re_, text = vals[0], vals[1]
            vectors["mat"].append({"name": name, "src": src, "re": re_.val, "text": text.as_bytes().hex(),
                                   "groups": [list(g) if g else None for g in vals[2:]]})
        elif kind == "matiter":
            re_, text = vals[0], vals[1]
            vectors["matiter"].append({"name": name, "src": src, "re": re_.val, "text": text.as_bytes().hex(),
                                       "matches": [list(g) for g in vals[2:]]})
        elif kind in ("matset", "nomatset"):
            res, text = vals[0], vals[1]
            vectors[kind].append({"name": name, "src": src, "res": [r.val for r in res],
                                  "text": text.as_bytes().hex(), "matches": vals[2:]})
        elif kind == "ismatch":
            vectors["ismatch"].append({"name": name, "src": src, "re": vals[0].val,
                                       "text": vals[1].as_bytes().hex(), "expect": vals[2]})
        elif kind == "noparse":
            vectors["noparse"].append({"name": name, "src": src, "re": vals[0].val})
        elif kind == "replace":  # tests/replace.rs:1-10
            which, (re_, text, rep, result) = raw[1].strip(), vals
            vectors["replace"].append({"name": name, "src": src, "which": which, "re": re_.val,
                                       "text": text.as_bytes().hex(), "mode": rep[0],
                                       "rep": rep[1].as_bytes().hex(), "result": result.as_bytes().hex()})
        elif kind == "expand":  # tests/macros_bytes.rs:26-38
            vectors["expand"].append({"name": name, "src": src, "re": vals[0].val, "text": vals[1].as_bytes().hex(),
                                      "template": vals[2].as_bytes().hex(), "result": vals[3].as_bytes().hex()})
        elif kind == "split":  # tests/macros.rs:140-149
            vectors["split"].append({"name": name, "src": src, "re": vals[0].val, "text": vals[1].as_bytes().hex(),
                                     "fields": [f[1].as_bytes().hex() for f in vals[2]]})


def bench_counts(path, macro, corpus):
    s = open(path, encoding="utf-8").read()
    out = []
    for m in re.finditer(r"(?m)^\s*%s!\(" % macro, s):
        prev = s[:m.start()].rstrip().rsplit("\n", 1)[-1].strip()
        # keep the answers of the Rust backend only (e.g. skip `#[cfg(feature = "re-re2")]`)
        if prev.startswith('#[cfg(feature = "re-') and "re-rust" not in prev:
            continue
        raw, _ = split_args(s, m.end())
        out.append({"name": raw[0], "re": parse_value(raw[1]).val, "count": int(raw[2]), "corpus": corpus,
                    "src": "%s:%d" % (os.path.relpath(path, REF), s.count("\n", 0, m.start()) + 1)})
    return out


def main():
    vectors = {k: [] for k in ("mat", "matiter", "matset", "nomatset", "ismatch", "noparse", "replace", "expand",
                               "split")}
    skipped = []
    for mod in MODULES:
        scan_file(os.path.join(REF, "tests", mod + ".rs"), vectors, skipped)
    scan_file(os.path.join(REF, "tests", "test_default_bytes.rs"), vectors, skipped)
    vectors["_about"] = ("Golden vectors of the reference regex 0.2.5 bytes::Regex test target "
                         "(tests/test_default_bytes.rs); texts are hex-encoded bytes; extracted by "
                         "tests/golden/extract_vectors.py")
    vectors["_skipped"] = skipped
    with open(os.path.join(OUT, "reference_vectors.json"), "w") as f:
        json.dump(vectors, f, indent=0, ensure_ascii=False)
    counts = bench_counts(os.path.join(REF, "bench/src/sherlock.rs"), "sherlock", "sherlock")
    # regexdna bench counts refer to bench/src/data/regexdna.txt which is absent
    # from this snapshot; the shootout known answer below covers the variants.
    dna_out = open(os.path.join(REF, "examples/regexdna-output.txt")).read().split("\n")
    variants = []
    for ln in dna_out[:9]:
        pat, cnt = ln.rsplit(" ", 1)
        variants.append({"re": pat, "count": int(cnt)})
    tail = [x for x in dna_out[9:] if x.strip()]
    known = {"sherlock": counts,
             "regexdna": {"src": "examples/regexdna-output.txt, examples/shootout-regex-dna-bytes.rs:21-64",
                          "strip": ">[^\n]*\n|\n", "variants": variants,
                          "input_len": int(tail[0]), "stripped_len": int(tail[1]), "substituted_len": int(tail[2])}}
    with open(os.path.join(OUT, "known_counts.json"), "w") as f:
        json.dump(known, f, indent=1)
    for src, dst in (("bench/src/data/sherlock.txt", "sherlock.txt.gz"),
                     ("examples/regexdna-input.txt", "regexdna-input.txt.gz")):
        data = open(os.path.join(REF, src), "rb").read()
        with gzip.GzipFile(os.path.join(OUT, dst), "wb", mtime=0) as g:
            g.write(data)
    n = {k: len(v) for k, v in vectors.items() if not k.startswith("_")}
    print("vectors:", n, "skipped:", len(skipped), "sherlock counts:", len(counts), file=sys.stderr)
    for s in skipped:
        print("  skipped", s, file=sys.stderr)


if __name__ == "__main__":
    main()
