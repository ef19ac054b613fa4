"""Loaders for the committed golden fixtures (tests/golden/)."""
import gzip
import json
import os

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def vectors():
    with open(os.path.join(G, "reference_vectors.json"), encoding="utf-8") as f:
        return json.load(f)


def known_counts():
    with open(os.path.join(G, "known_counts.json")) as f:
        return json.load(f)


def corpus(name):
    fn = {"sherlock": "sherlock.txt.gz", "regexdna": "regexdna-input.txt.gz"}[name]
    with gzip.open(os.path.join(G, fn), "rb") as f:
        return f.read()


def stdlib_fixtures():
    """Python-`re` answers for the BASELINE patterns (gen_stdlib_fixtures.py)."""
    with gzip.open(os.path.join(G, "stdlib_re_fixtures.json.gz"), "rt", encoding="ascii") as f:
        return json.load(f)


def stdlib_looks_fixtures():
    """Python-`re` finditer answers for look-around regexes over ASCII slices
    of the sherlock corpus (gen_stdlib_looks.py); returns (fixtures, text)."""
    with gzip.open(os.path.join(G, "stdlib_looks_fixtures.json.gz"), "rt", encoding="ascii") as f:
        fx = json.load(f)
    return fx, bytes(b if b < 0x80 else 0x20 for b in corpus("sherlock"))
