#!/usr/bin/env python3
"""Extract regex-syntax's literal-extraction test vectors as JSON data.

Reads (as text, in the build container) the declarative tests at the end of
the reference's regex-syntax/src/literals.rs — test_lit! (prefixes /
suffixes of a pattern with the default limits), test_exhausted! (limits 20
bytes / 10 class members), test_unamb! (unambiguous_prefixes), test_lcp! and
test_lcs! — and writes tests/golden/literal_vectors.json.  Expected literals
keep the tests' own escaped form (Rust escape_default per byte, 'M' =
complete, 'C' = cut).  Only inputs and expected outputs are written (data).
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from extract_vectors import parse_string, split_args  # noqa: E402

SRC = "/root/reference/regex-syntax/src/literals.rs"


def lit_list(args):
    out = []
    for a in args:
        a = a.strip()
        m = re.match(r"^([MC])\((.*)\)$", a, re.S)
        assert m, a
        lit, _ = parse_string(m.group(2).strip(), 0)
        out.append([m.group(1), lit.val])
    return out


def vec_arg(a):
    a = a.strip()
    assert a.startswith("vec!["), a
    inner = a[5:]
    args, _ = split_args(inner.replace("]", ")", 1) if False else inner[:-1] + ")", 0)
    return args


def main():
    s = open(SRC).read()
    s = s[s.index("mod tests"):]
    out = {"lit": [], "exhausted": [], "unamb": [], "lcp": [], "lcs": []}
    for m in re.finditer(r"\b(test_lit|test_exhausted|test_unamb|test_lcp|test_lcs)!\(", s):
        if s[m.start() - 15:m.start()].strip().endswith("macro_rules!"):
            continue
        args, _ = split_args(s, m.end())
        kind = m.group(1)
        if args and args[0].startswith("$"):
            continue  # the macro definitions themselves
        if kind in ("test_lit", "test_exhausted"):
            name, which, pat = args[0], args[1], parse_string(args[2].strip(), 0)[0].val
            out["lit" if kind == "test_lit" else "exhausted"].append(
                {"name": name, "which": which, "re": pat, "expected": lit_list(args[3:])})
        elif kind == "test_unamb":
            out["unamb"].append({"name": args[0], "given": lit_list(vec_arg(args[1])),
                                 "expected": lit_list(vec_arg(args[2]))})
        else:
            given = [parse_string(a.strip(), 0)[0].val for a in vec_arg(args[1])]
            out[kind[5:]].append({"name": args[0], "given": given,
                                  "expected": parse_string(args[2].strip(), 0)[0].val})
    with open(os.path.join(HERE, "literal_vectors.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print({k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
