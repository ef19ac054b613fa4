"""replace / split on the GPU against the reference's replace!/expand!/split!
vectors and its documentation examples (re_bytes.rs), against the oracle
restatement (tests/replace_ref.py) on seeded inputs, batched, and the
regex-dna pipeline's known answers (examples/regexdna-output.txt)."""
import zlib

import numpy as np
import pytest

import regex_amd as R
from golden_data import corpus, known_counts, vectors
from oracle_py import OracleRegex
import replace_ref as RR

pytestmark = pytest.mark.gpu

V = vectors()


@pytest.mark.parametrize("v", V["replace"], ids=[x["name"] for x in V["replace"]])
def test_replace_vectors(cuda, v):
    re = R.Regex(v["re"])
    text, rep = bytes.fromhex(v["text"]), bytes.fromhex(v["rep"])
    if v["mode"] == "literal":
        rep = R.NoExpand(rep)
    got = re.replace(text, rep) if v["which"] == "replace" else re.replace_all(text, rep)
    assert got == bytes.fromhex(v["result"]), v["src"]


@pytest.mark.parametrize("v", V["expand"], ids=[x["name"] for x in V["expand"]])
def test_expand_vectors(cuda, v):
    re = R.Regex(v["re"])
    text = bytes.fromhex(v["text"])
    g = re.captures(text)
    assert R.expand(g, re.capture_names(), bytes.fromhex(v["template"]), text) == bytes.fromhex(v["result"])


@pytest.mark.parametrize("v", V["split"], ids=[x["name"] for x in V["split"]])
def test_split_vectors(cuda, v):
    assert R.Regex(v["re"]).split(bytes.fromhex(v["text"])) == [bytes.fromhex(f) for f in v["fields"]]


def test_doc_examples(cuda):
    """The examples in re_bytes.rs's documentation of split/splitn/replace."""
    assert R.Regex(r"[ \t]+").split(b"a b \t  c\td    e") == [b"a", b"b", b"c", b"d", b"e"]
    assert R.Regex(r"\W+").splitn(b"Hey! How are you?", 3) == [b"Hey", b"How", b"are you?"]
    assert R.Regex("[^01]+").replace(b"1078910", b"") == b"1010"
    re = R.Regex(r"([^,\s]+),\s+(\S+)")
    assert re.replace(b"Springsteen, Bruce", lambda g, t: t[g[2][0]:g[2][1]] + b" " + t[g[1][0]:g[1][1]]) \
        == b"Bruce Springsteen"
    re = R.Regex(r"(?P<last>[^,\s]+),\s+(?P<first>\S+)")
    assert re.replace(b"Springsteen, Bruce", b"$first $last") == b"Bruce Springsteen"
    re = R.Regex(r"(?P<first>\w+)\s+(?P<second>\w+)")
    assert re.replace(b"deep fried", b"${first}_$second") == b"deep_fried"
    re = R.Regex(r"(?P<last>[^,\s]+),\s+(\S+)")
    assert re.replace(b"Springsteen, Bruce", R.NoExpand(b"$2 $last")) == b"$2 $last"


PATS = [r"\d+", r"a*", r"", r"\b", r"x|yz", r"(\w)(\d)?", r"[ \t]+", r"^", r"$", r"(?m)^\w"]
ALPHA = [b"a", b"b", b"x", b"y", b"z", b"1", b"2", b" ", b"\t", b"\n", "é".encode()]


def _texts(seed, n, hi=30):
    import random
    rng = random.Random(seed)
    return [b"".join(rng.choice(ALPHA) for _ in range(rng.randint(0, hi))) for _ in range(n)]


@pytest.mark.parametrize("pat", PATS)
def test_single_vs_oracle(cuda, pat):
    re = R.Regex(pat)
    o = OracleRegex(re)
    names = re.capture_names()
    for t in _texts(zlib.crc32(pat.encode()), 40):
        for rep, lit in ((b"<$1>", False), (b"-", True), (b"", True)):
            for limit in (0, 1, 2):
                exp = RR.replacen(o, names, t, limit, rep, lit)
                got = re.replacen(t, limit, R.NoExpand(rep) if lit else rep)
                assert got == exp, (pat, t, rep, limit)
        assert re.split(t) == RR.split(o, t), (pat, t)
        for n in range(5):
            assert re.splitn(t, n) == RR.splitn(o, t, n), (pat, t, n)


def ragged(texts):
    offs = np.zeros(len(texts) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(t) for t in texts])
    buf = np.frombuffer(b"".join(texts) + b"\0" * 16, dtype=np.uint8).copy()
    return buf, offs


@pytest.mark.parametrize("pat", PATS)
@pytest.mark.parametrize("limit", [0, 1, 3])
def test_replace_batch_vs_oracle(cuda, pat, limit):
    import torch
    re = R.Regex(pat)
    o = OracleRegex(re)
    texts = _texts(zlib.crc32(pat.encode()) + limit, 300, 60)
    buf, offs = ragged(texts)
    for rep in (b"", b"<->", b"$1"):
        out, ooff = re.replace_batch(torch.from_numpy(buf).to(cuda), rep, limit=limit,
                                     offsets=torch.from_numpy(offs).to(cuda))
        out = out.cpu().numpy().tobytes()
        ooff = ooff.cpu().numpy()
        for i, t in enumerate(texts):
            exp = RR.replacen(o, None, t, limit, rep, True)
            assert out[ooff[i]:ooff[i + 1]] == exp, (pat, t, rep, limit)


@pytest.mark.parametrize("pat", PATS)
@pytest.mark.parametrize("limit", [None, 0, 1, 2, 3])
def test_split_batch_vs_oracle(cuda, pat, limit):
    import torch
    re = R.Regex(pat)
    o = OracleRegex(re)
    texts = _texts(zlib.crc32(pat.encode()) + 7, 300, 60)
    buf, offs = ragged(texts)
    counts, pieces = re.split_batch(torch.from_numpy(buf).to(cuda), limit=limit,
                                    offsets=torch.from_numpy(offs).to(cuda))
    counts = counts.cpu().numpy()
    pieces = pieces.cpu().numpy()
    k = 0
    for i, t in enumerate(texts):
        exp = RR.split(o, t) if limit is None else RR.splitn(o, t, limit)
        got = [t[a:b] for a, b in pieces[k:k + counts[i]]]
        k += counts[i]
        assert got == exp, (pat, t, limit)
    assert k == len(pieces)


def test_replace_batch_strided_long(cuda):
    """Fixed-stride long haystacks (the chunked find_iter path) with dense
    matches: output layout and bytes against the oracle."""
    import torch
    from regex_amd.workloads import date_haystacks_host
    n, L = 64, 1 << 16
    buf, _ = date_haystacks_host(n, L, seed=3, frac=0.5)
    re = R.Regex(r"\d+")
    o = OracleRegex(re)
    out, ooff = re.replace_batch(torch.from_numpy(buf).to(cuda), b"#", stride=L, length=L, count=n)
    out = out.cpu().numpy().tobytes()
    ooff = ooff.cpu().numpy()
    for i in range(0, n, 7):
        t = bytes(buf[i * L:(i + 1) * L])
        assert out[ooff[i]:ooff[i + 1]] == RR.replacen(o, None, t, 0, b"#", True), i


# examples/shootout-regex-dna-bytes.rs:41-53 (IUB codes -> alternatives)
SUBSTS = [("B", b"(c|g|t)"), ("D", b"(a|g|t)"), ("H", b"(a|c|t)"), ("K", b"(g|t)"), ("M", b"(a|c)"),
          ("N", b"(a|c|g|t)"), ("R", b"(a|g)"), ("S", b"(c|g)"), ("V", b"(a|c|g)"), ("W", b"(a|t)"),
          ("Y", b"(c|t)")]


@pytest.mark.parametrize("copies", [1, 64])
def test_regexdna_pipeline(cuda, copies):
    """The shootout pipeline end to end on the GPU: strip, variant counts,
    IUB substitutions; lengths and counts from examples/regexdna-output.txt."""
    import torch
    kc = known_counts()["regexdna"]
    one = corpus("regexdna")
    L = len(one)
    assert L == kc["input_len"]
    hay = torch.from_numpy(np.frombuffer(one * copies + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    seq, soff = R.Regex(kc["strip"]).replace_batch(hay, b"", stride=L, length=L, count=copies)
    soff_h = soff.cpu().numpy()
    assert all(soff_h[i + 1] - soff_h[i] == kc["stripped_len"] for i in range(copies))
    seq = torch.cat([seq, torch.zeros(16, dtype=torch.uint8, device=cuda)])
    for v in kc["variants"]:
        counts, _ = R.Regex(v["re"]).find_iter_batch(seq, offsets=soff)
        assert counts.cpu().numpy().tolist() == [v["count"]] * copies, v["re"]
    cur, coff = seq, soff
    for pat, rep in SUBSTS:
        cur, coff = R.Regex(pat).replace_batch(cur, rep, offsets=coff)
        cur = torch.cat([cur, torch.zeros(16, dtype=torch.uint8, device=cuda)])
    coff_h = coff.cpu().numpy()
    assert all(coff_h[i + 1] - coff_h[i] == kc["substituted_len"] for i in range(copies))
