"""Host side of the Shift-And find_iter engine (build.cpp build_shiftand,
used by iter_spec_sa_kernel): the class sequences merged from a string set
must recognise exactly the set.  The automaton is stepped here as the kernel
steps it (D = ((D << 1) | init) & mask[b]; a final bit after byte q = a string
ending at q) and compared with brute-force occurrences of every string, on
random texts over the strings' own bytes.  No GPU needed."""
import random
import zlib

import pytest

import regex_amd as R

PATTERNS = [r"agggtaaa|tttaccct", r"[cgt]gggtaaa|tttaccc[acg]", r"agggt[cgt]aa|tt[acg]accct", r"aa", r"e",
            r"(?i)holm", r"Holmes|Watson", r"[0-3]{2}", r"abc|abd", r"é", r"x(ab|cd)y", r"aaaaaaa",
            r"(?i)the", r"ab|cd|ef|gh"]


def ends_sa(img, text):
    bits, mask, init, fin, L = img
    full = (1 << 64) - 1
    D, out = 0, []
    for q, b in enumerate(text):
        D = (((D << 1) | init) & full) & mask[b]
        if D & fin:
            out.append(q)
    return out


def ends_brute(lits, text):
    return sorted(set(i + len(l) - 1 for l in lits for i in range(len(text) - len(l) + 1)
                      if text[i:i + len(l)] == l))


@pytest.mark.parametrize("pat", PATTERNS)
def test_shiftand_image_recognises_the_set(pat):
    re = R.Regex(pat)
    lits = re.literals()
    img = re.shiftand()
    assert img is not None, pat
    bits, mask, init, fin, L = img
    assert all(len(l) == L for l in lits) and bits % L == 0 and bits <= 64
    assert bin(init).count("1") == bits // L == bin(fin).count("1")
    rng = random.Random(zlib.crc32(pat.encode()))
    alphabet = sorted(set(b for l in lits for b in l)) + [ord("z")]
    for _ in range(20):
        parts = [rng.choice(lits) if rng.random() < 0.3 else bytes([rng.choice(alphabet)]) for _ in range(200)]
        text = b"".join(parts)
        assert ends_sa(img, text) == ends_brute(lits, text), pat


def test_shiftand_merges_classes():
    # the six strings of a regex-dna variant merge into two class sequences
    assert R.Regex(r"[cgt]gggtaaa|tttaccc[acg]").shiftand()[0] == 16
    assert R.Regex(r"(?i)holm").shiftand()[0] == 4
    assert R.Regex(r"[0-3]{2}").shiftand()[0] == 2


def test_shiftand_absent():
    assert R.Regex(r"Sherlock|Holmes").shiftand() is None  # unequal lengths
    assert R.Regex(r"a+").shiftand() is None               # not a finite set
