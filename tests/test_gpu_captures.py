"""Captures on the GPU (rure_find_captures / rure_amd_captures_batch: DFA
bounds, then the captures Pike VM kernel) against the oracle's
read_captures_at (exec.rs:524-596 restated) and the reference's golden
groups."""
import zlib

import numpy as np
import pytest

import regex_amd as R
from golden_data import vectors
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

V = vectors()


def ragged(texts):
    offs = np.zeros(len(texts) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(t) for t in texts])
    buf = np.frombuffer(b"".join(texts) + b"\0" * 16, dtype=np.uint8).copy()
    return buf, offs


def rows(t, n):
    out = []
    for i in range(n):
        a, b = int(t[i, 0]), int(t[i, 1])
        out.append(None if a < 0 or b < 0 else (a, b))
    return out


def test_golden_groups_batched(cuda):
    """Every `mat!` vector: one batched call per pattern, groups as the
    reference's tests expect (and as the oracle's dispatch gives)."""
    import torch
    bad = []
    for v in V["mat"]:
        re = R.Regex(v["re"])
        t = bytes.fromhex(v["text"])
        buf, offs = ragged([t])
        got = re.captures_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda))
        g = rows(got[0].cpu().numpy(), re.captures_len())
        exp = [tuple(x) if x else None for x in v["groups"]]
        g = None if g[0] is None else g
        o = OracleRegex(re).captures(t)
        if g != o or (g is None and exp != [None]) or (g is not None and g[:len(exp)] != exp):
            bad.append((v["name"], g, o, exp))
    assert not bad, bad[:5]


def test_golden_groups_single_call(cuda):
    for v in V["mat"][:120]:
        re = R.Regex(v["re"])
        t = bytes.fromhex(v["text"])
        assert re.captures(t) == OracleRegex(re).captures(t), v["name"]


CAP_PATTERNS = [
    r"(a)(b)?(c)", r"(?P<y>\d{4})-(?P<m>\d{2})-(?P<d>\d{2})", r"(a|ab)(c|bcd)(d*)", r"((a)|b)+",
    r"(a*)+", r"(a*)*b", r"(a+|b+)*c", r"(?:(a)|(b))*", r"(a??)(a*?)", r"(a?)+b", r"(a|b?)+c",
    r"(\w+)@(\w+)\.(\w+)", r"(?m)^(\w+) (\w+)$", r"(a..$)|(a)", r"(ab|a)(bc|c)?$", r"(x)(?-u:\b)",
    r"(?i)(stra)(ss|ß)e", r"([0-9]+)(\.[0-9]+)?", r"(a)|(b)|(c)", r"((((a))))", r"(.)(.)(.)(.)(.)",
    r"^(a+)(b*)", r"(a+)(b*)$", r"\b(\w+)\b", r"(\w)\B(\w)", r"(?-u:\b)(a+)",
]
ALPHABET = [b"a", b"b", b"c", b"d", b"x", b"1", b".", b" ", b"\n", b"@", b"s", "ß".encode(), "é".encode(),
            b"\xff"]


def _texts(seed, n, hi=40):
    import random
    rng = random.Random(seed)
    return [b"".join(rng.choice(ALPHABET) for _ in range(rng.randint(0, hi))) for _ in range(n)]


@pytest.mark.parametrize("pat", CAP_PATTERNS)
@pytest.mark.parametrize("start", [0, 3])
def test_captures_batch_vs_oracle(cuda, pat, start):
    import torch
    re = R.Regex(pat)
    o = OracleRegex(re)
    texts = _texts(zlib.crc32(pat.encode()) + start, 400)
    buf, offs = ragged(texts)
    got = re.captures_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda),
                            start=start).cpu().numpy()
    ng = re.captures_len()
    for i, t in enumerate(texts):
        g = rows(got[i], ng)
        g = None if g[0] is None else g
        exp = o.captures(t, start) if start <= len(t) else None
        assert g == exp, (pat, t, start, g, exp)


def test_captures_strided_dates(cuda):
    """Fixed-stride batch (the C2 layout) with date groups."""
    import torch
    from regex_amd.workloads import date_haystacks_host
    n, L = 2048, 256
    buf, _ = date_haystacks_host(n, L, seed=5, frac=0.4)
    re = R.Regex(r"(?P<y>\d{4})-(?P<m>\d{2})-(?P<d>\d{2})")
    o = OracleRegex(re)
    got = re.captures_batch(torch.from_numpy(buf).to(cuda), stride=L, length=L, count=n).cpu().numpy()
    for i in range(n):
        g = rows(got[i], 4)
        g = None if g[0] is None else g
        assert g == o.captures(bytes(buf[i * L:(i + 1) * L])), i


def test_captures_scratch_path(cuda):
    """A program whose per-wave slot rows exceed LDS (global scratch path)."""
    import torch
    re = R.Regex(r"(\w+) (\w+) (\w+) (\w+) (\w+)")
    info = re.nfa_tables()[0]
    ns = 2 * re.captures_len()
    assert info["leaves"] * (16 * ns + 12) > 160 * 1024
    o = OracleRegex(re)
    texts = [("héllo wörld foo bar baz qux " * k).encode() for k in range(1, 6)] + _texts(77, 60, 80)
    buf, offs = ragged(texts)
    got = re.captures_batch(torch.from_numpy(buf).to(cuda), offsets=torch.from_numpy(offs).to(cuda)).cpu().numpy()
    for i, t in enumerate(texts):
        g = rows(got[i], 6)
        g = None if g[0] is None else g
        assert g == o.captures(t), t


def test_captures_iter_vs_oracle(cuda):
    import replace_ref as RR
    for pat, t in ((r"(\w)(\d)?", b"a1 b c22 d" * 3 + "\u00e93".encode()),
                   (r"\b", b"\nb1ybby2\n y\nb" + "\u00e9\u00e9".encode() + b"y")):
        re = R.Regex(pat)
        assert re.captures_iter(t) == RR.captures_iter(OracleRegex(re), t), pat


def rure_iter_oracle(o, t, caps=False):
    """regex-capi/src/rure.rs:322-397 over the oracle."""
    out, last_end, last_match = [], 0, None
    while last_end <= len(t):
        g = o.captures(t, last_end) if caps else o.find(t, last_end)
        if g is None:
            break
        s, e = g[0] if caps else g
        if s == e:
            last_end += 1
            if last_match == e:
                continue
        else:
            last_end = e
        last_match = e
        out.append(g)
    return out


def test_c_api_iteration_differs_from_find_iter(cuda):
    """After an empty match rure_iter_next restarts one past the previous
    search start, not past the match: with a Unicode word boundary next to
    non-ASCII bytes (the DFA reads only the byte before the start) it revisits
    an earlier position, which find_iter never does.  Both reproduced."""
    t = b"\nb1ybby2\n y\nb" + "\u00e9\u00e9".encode() + b"y"
    re = R.Regex(r"\b")
    o = OracleRegex(re)
    assert re.find_iter(t) == o.find_iter(t)
    assert re.iter_rure(t) == rure_iter_oracle(o, t)
    assert re.captures_iter_rure(t) == rure_iter_oracle(o, t, caps=True)
    assert re.iter_rure(t)[-3:] == [(18, 18), (17, 17), (18, 18)]
    assert re.find_iter(t)[-1] == (18, 18) and (17, 17) not in re.find_iter(t)


def test_reference_quirk_on_gpu(cuda):
    re = R.Regex(r"(a..$)|(a)")
    assert re.find(b"abcd") == (0, 1)
    assert re.captures(b"abcd") == [(0, 3), (0, 3), None]


def test_empty_and_one_group(cuda):
    import torch
    re = R.Regex(r"a+")
    assert re.captures_len() == 1
    assert re.captures(b"xaay") == [(1, 3)]
    dev = torch.zeros(16, dtype=torch.uint8, device=cuda)
    assert re.captures_batch(dev, stride=4, length=4, count=0).shape == (0, 1, 2)
    assert R.Regex(r"(a)|b").captures(b"") is None
