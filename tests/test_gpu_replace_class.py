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
