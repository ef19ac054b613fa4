"""replace_all of a one-byte-class regex on the GPU without a match list
(replace_scan.hip launch_replace_class, last_fwd_path -23) against the
oracle's find_iter + the reference's replacen rule (re_bytes.rs:489-512):
sparse, dense and all-class text, replacements of 1 to 64 bytes, lengths
around the 64-byte lane and 4 KiB unit edges, an output buffer smaller than
the result (the call reports the length, the retry writes it), and the
regex-dna IUB substitutions chained (their known output length)."""
import ctypes
import random

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu


def dev(t, cuda):
    import torch
    return torch.from_numpy(np.frombuffer(t + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)


def expect(re, t, rep):
    out, last = bytearray(), 0
    for s, e in OracleRegex(re).find_iter(t):
        out += t[last:s] + rep
        last = e
    return bytes(out + t[last:])


def text(seed, n, alpha):
    rng = random.Random(seed)
    return bytes(rng.choice(alpha) for _ in range(n))


CASES = [(r"B", b"acgtB"), (r"[KM]", b"acgtacgtacgtKM"), (r"x", b"x"), (r"[a-c]", b"abcdefgh \n"),
         (r"(?-u)\xff", b"a\xff\xfe"), (r"(?s-u:.)", b"ab\n")]


@pytest.mark.parametrize("pat,alpha", CASES)
@pytest.mark.parametrize("n", [0, 1, 15, 63, 64, 65, 4095, 4096, 4097, 70001])
@pytest.mark.parametrize("rep", [b"Z", b"(c|g|t)", b"<" + b"r" * 62 + b">"])
def test_replace_class(cuda, pat, alpha, n, rep):
    re = R.Regex(pat)
    t = text(n * 7 + len(rep), n, alpha)
    out, ooff = re.replace_batch(dev(t, cuda), rep, stride=max(n, 1), length=n, count=1)
    if n:
        assert N.rure_amd_last_fwd_path() == -23
    assert bytes(out.cpu().numpy()) == expect(re, t, rep), (pat, n, rep)
    assert ooff.cpu().numpy().tolist() == [0, len(expect(re, t, rep))]


def test_replace_class_small_buffer(cuda):
    """An output buffer shorter than the result: *total is the length and no
    byte past the capacity is written."""
    import torch
    re = R.Regex(r"[KM]")
    t = text(5, 50000, b"acgtKM")
    exp = expect(re, t, b"(a|c)")
    d = dev(t, cuda)
    b = R._batch(d, None, len(t), len(t), 1, 0)
    cap = len(exp) // 3
    out = torch.full((cap + 64,), 0xAB, dtype=torch.uint8, device=cuda)
    ooff = torch.empty(2, dtype=torch.int64, device=cuda)
    total = torch.zeros(1, dtype=torch.int64, device=cuda)
    rc = N.rure_amd_replace_batch(re._re, ctypes.byref(b), b"(a|c)", 5, 0, ctypes.c_void_p(out.data_ptr()),
                                  ctypes.c_void_p(ooff.data_ptr()), cap, ctypes.c_void_p(total.data_ptr()),
                                  R._stream_ptr(None))
    assert rc == N.OK
    torch.cuda.synchronize()
    assert int(total.item()) == len(exp)
    got = out.cpu().numpy()
    assert bytes(got[:cap]) == exp[:cap]
    assert (got[cap:] == 0xAB).all()


def test_iub_chain_known_length(cuda):
    """The 11 IUB substitutions of the regex-dna shootout chained over the
    stripped input: the output length the reference prints."""
    from golden_data import corpus, known_counts
    from regex_amd import shootout
    kc = known_counts()["regexdna"]
    raw = corpus("regexdna")
    strip = R.Regex(shootout.STRIP.decode())
    seq = strip.replace_all(raw, b"")
    cur = dev(seq, cuda)
    n = len(seq)
    for p, rep in shootout.SUBSTS:
        re = R.Regex(p.decode())
        out, ooff = re.replace_batch(cur, rep, stride=n, length=n, count=1)
        assert N.rure_amd_last_fwd_path() == -23
        n = int(ooff[1].item())
        import torch
        cur = torch.cat([out[:n], torch.zeros(16, dtype=torch.uint8, device=cuda)])
    assert n == kc["substituted_len"], (n, kc["substituted_len"])


def chain_expect(steps, t):
    for re, rep in steps:
        t = expect(re, t, rep)
    return t


CHAINS = [
    # the IUB substitutions' shape: one byte each, the next step's byte counted as written
    [(r"B", b"(c|g|t)"), (r"D", b"(a|g|t)"), (r"N", b"(a|c|g|t)")],
    # two-byte classes (SWAR), a wide class (the count pass), a 64-byte replacement
    [(r"[KM]", b"<km>"), (r"[a-c]", b"Q"), (r"Q", b"<" + b"q" * 62 + b">"), (r"[<>]", b"D")],
    # replacements that create the next step's bytes, and a one-step chain
    [(r"x", b"yxy"), (r"y", b"xx")],
    [(r"(?-u)\xff", b"\xff\xfe\xff")],
]


@pytest.mark.parametrize("seq", [0, 1])
@pytest.mark.parametrize("ci", range(len(CHAINS)))
@pytest.mark.parametrize("n", [0, 1, 63, 4096, 4097, 70001, 300007])
def test_replace_chain(cuda, knobs, seq, ci, n):
    """rure_amd_replace_all_chain against the host rule applied step by step:
    the same bytes and every intermediate length — as one composed byte map
    (default, last_fwd_path -24) and step by step (knob chain_seq=1, -23)."""
    if seq:
        knobs(chain_seq=1)
    steps = [(R.Regex(p), rep) for p, rep in CHAINS[ci]]
    alpha = b"acgtBDNKMxy\xff\xfe<>Q\n"
    t = text(ci * 1000 + n, n, alpha)
    out, lengths = R.replace_all_chain([r for r, _ in steps], [rep for _, rep in steps], dev(t, cuda), length=n,
                                       capacity=16 * n + 4096)
    exp, lens = t, [n]
    for re, rep in steps:
        exp = expect(re, exp, rep)
        lens.append(len(exp))
    assert lengths.cpu().numpy().tolist() == lens
    assert bytes(out[:lens[-1]].cpu().numpy()) == exp
    if n:
        assert N.rure_amd_last_fwd_path() == (-23 if seq else -24)


@pytest.mark.parametrize("seq", [0, 1])
def test_replace_chain_cut(cuda, knobs, seq):
    """A capacity below an intermediate length: that step's length is exact,
    the later ones are at least as large (step by step they are lower bounds:
    a step reads its input cut), so lengths[-1] > capacity and the caller
    retries with it until the chain fits."""
    if seq:
        knobs(chain_seq=1)
    steps = [(R.Regex(r"x"), b"x" * 40), (R.Regex(r"y"), b"yy"), (R.Regex(r"z"), b"zzz")]
    t = text(5, 20000, b"xyz ")
    exps = [t]
    for re, rep in steps:
        exps.append(expect(re, exps[-1], rep))
    cap, tries = len(t) + 100, 0
    while True:
        out, lengths = R.replace_all_chain([r for r, _ in steps], [rep for _, rep in steps], dev(t, cuda),
                                           length=len(t), capacity=cap)
        ln = lengths.cpu().numpy().tolist()
        tries += 1
        assert ln[0] == len(t) and ln[1] == len(exps[1]) and ln[1] <= ln[2] <= ln[3]
        if ln[3] <= cap:
            break
        assert ln[3] > cap
        cap = ln[3]
    assert tries >= 2
    assert ln == [len(x) for x in exps]
    assert bytes(out[:ln[3]].cpu().numpy()) == exps[3]


def test_replace_chain_rejects(cuda):
    """A regex whose matches are not single class bytes is refused."""
    with pytest.raises(Exception):
        R.replace_all_chain([R.Regex(r"ab")], [b"x"], dev(b"abab", cuda), length=4)


def test_replace_chain_long_images(cuda):
    """Images longer than 64 bytes after composition (x -> 40 x, then each x
    -> 2 x): the call runs the chain step by step (-23), same bytes."""
    steps = [(R.Regex(r"x"), b"x" * 40), (R.Regex(r"x"), b"xx")]
    t = text(9, 5000, b"xab")
    out, lengths = R.replace_all_chain([r for r, _ in steps], [rep for _, rep in steps], dev(t, cuda), length=len(t),
                                       capacity=100 * len(t))
    assert N.rure_amd_last_fwd_path() == -23
    exp = chain_expect(steps, t)
    assert int(lengths[-1]) == len(exp)
    assert bytes(out[:len(exp)].cpu().numpy()) == exp
