"""GPU parity of rure_amd_find_iter_span_multi (regex_amd.find_iter_span_multi):
several regexes over one span in one pass.  Each regex's count, matches and
exit must be exactly its own find_iter_span's (re_trait.rs:197-221), for the
regex-dna variants (one fused Shift-And pass), chained spans entered with the
previous span's exits, text dense in matches (repairs at unit cuts), and
lists that cannot be fused (the per-regex fallback)."""
import numpy as np
import pytest

import regex_amd as R
from golden_data import corpus, known_counts
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu


def dev(buf, cuda):
    import torch
    t = torch.zeros(len(buf) + 16, dtype=torch.uint8)
    t[: len(buf)] = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy())
    return t.to(cuda)


def pairs(m):
    return [(int(a), int(b)) for a, b in m.cpu().numpy()]


def variants():
    return [R.Regex(v["re"]) for v in known_counts()["regexdna"]["variants"]]


def stripped(copies):
    kc = known_counts()["regexdna"]
    seq = R.Regex(kc["strip"]).replace_all(corpus("regexdna"), b"")
    return seq * copies


def check_same(res, h, n, lo, hi, entries=None):
    got = R.find_iter_span_multi(res, h, lo, hi, length=n, entries=entries)
    for i, re in enumerate(res):
        c, m, x = re.find_iter_span(h, lo, hi, length=n, entry=None if entries is None else entries[i])
        assert int(got[i][0].item()) == int(c.item()), (i, lo, hi)
        assert pairs(got[i][1]) == pairs(m), (i, lo, hi)
        assert got[i][2].tolist() == x.tolist(), (i, lo, hi)
    return got


def test_multi_variants_whole(cuda):
    seq = stripped(6)
    res = variants()
    h = dev(seq, cuda)
    got = check_same(res, h, len(seq), 0, len(seq))
    for i, re in enumerate(res):  # and the oracle's find_iter
        assert pairs(got[i][1]) == OracleRegex(re).find_iter(seq), i


def test_multi_variants_spans_chained(cuda):
    seq = stripped(3)
    res = variants()
    h = dev(seq, cuda)
    n = len(seq)
    cuts = [0, n // 3 + 5, n // 2 + 1, n]
    entries = None
    for lo, hi in zip(cuts, cuts[1:]):
        got = check_same(res, h, n, lo, hi, entries)
        entries = [g[2] for g in got]


def test_multi_dense_matches(cuda):
    # matches everywhere and across every unit cut: repairs must agree
    rng = np.random.default_rng(5)
    motifs = [b"agggtaaa", b"tttaccct", b"cgggtaaa", b"tttacccg", b"aggggtaa"]
    parts = [motifs[int(i)] if rng.random() < 0.5 else bytes(rng.choice(np.frombuffer(b"acgt", dtype=np.uint8), size=int(rng.integers(1, 9))))
             for i in rng.integers(0, len(motifs), size=200000)]
    text = b"".join(parts)
    res = variants()
    h = dev(text, cuda)
    check_same(res, h, len(text), 0, len(text))
    check_same(res, h, len(text), 7, len(text) - 3)


def test_multi_not_fusable(cuda):
    # mixed engines / lengths: each regex runs its own pass, same results
    seq = stripped(2)
    res = variants()[:3] + [R.Regex(r"a+"), R.Regex(r"agg|tttaccct")]
    h = dev(seq, cuda)
    check_same(res, h, len(seq), 0, len(seq))


@pytest.mark.parametrize("k", [1, 2, 4, 9])
def test_multi_counts_known_answers(cuda, k):
    kc = known_counts()["regexdna"]
    seq = stripped(1)
    res = variants()[:k]
    h = dev(seq, cuda)
    got = R.find_iter_span_multi(res, h, 0, len(seq), length=len(seq))
    for i in range(k):
        assert int(got[i][0].item()) == kc["variants"][i]["count"], i


@pytest.mark.parametrize("engine", ["kmer", "shiftand"])
def test_multi_engines_mixed_bytes(cuda, knobs, engine):
    """The fused pass with the k-mer probe engine (default for the regex-dna
    variants) and with the Shift-And words (knob kmer=0): text with
    uppercase ACGT, IUB codes, 'n', bytes >= 0x80 and newlines between the
    motifs — every regex's output equals its own single pass and the oracle."""
    if engine == "shiftand":
        knobs(kmer=0)
    rng = np.random.default_rng(11)
    motifs = [b"agggtaaa", b"tttaccct", b"cgggtaaa", b"tttacccg", b"aggggtaa", b"ggtaaaTT", b"AGGGTAAA"]
    noise = np.frombuffer(b"acgtacgtACGTnNBDHKMRSVWY\n\x80\xff\xc3\xa9", dtype=np.uint8)
    parts = [motifs[int(i)] if rng.random() < 0.4 else bytes(rng.choice(noise, size=int(rng.integers(1, 12))))
             for i in rng.integers(0, len(motifs), size=150000)]
    text = b"".join(parts)
    res = variants()
    h = dev(text, cuda)
    got = check_same(res, h, len(text), 0, len(text))
    for i, re in enumerate(res):
        assert pairs(got[i][1]) == OracleRegex(re).find_iter(text), i
    check_same(res, h, len(text), 13, len(text) - 5)


def test_multi_kmer_known_answers(cuda):
    """The regex-dna known answers through the k-mer engine over many copies."""
    kc = known_counts()["regexdna"]
    seq = stripped(40)
    res = variants()
    h = dev(seq, cuda)
    got = R.find_iter_span_multi(res, h, 0, len(seq), length=len(seq))
    one = stripped(1)
    for v, re, g in zip(kc["variants"], res, got):
        seam = len(OracleRegex(re).find_iter(one * 2)) - 2 * v["count"]
        assert int(g[0].item()) == v["count"] * 40 + seam * 39, v["re"]


@pytest.mark.parametrize("extra", [0, 1])
def test_multi_kmer_many_codes(cuda, extra):
    """String sets whose codes admit no injective 10-bit hash (192 and 256
    8-byte strings over acgt, above the 160 the search is tried for): the
    k-mer engine settles its hits through the global mask table instead of
    the LDS hash, with outputs equal to each regex's own pass and the oracle."""
    pats = [r"[acgt]{3}ggtaa", r"tt[acgt]{3}acc", r"cc[acgt]{3}tgg"] + ([r"a[acgt]{3}tgca"] if extra else [])
    res = [R.Regex(p) for p in pats]
    rng = np.random.default_rng(21 + extra)
    text = bytes(rng.choice(np.frombuffer(b"acgt", dtype=np.uint8), size=400000))
    h = dev(text, cuda)
    got = check_same(res, h, len(text), 0, len(text))
    for i, re in enumerate(res):
        exp = OracleRegex(re).find_iter(text)
        assert len(exp) > 100
        assert pairs(got[i][1]) == exp, i
