"""GPU parity of the sharded find_iter (rure_amd_find_iter_span +
regex_amd.dist's exit exchange): a haystack cut into k spans,
each iterated on the device from a fresh start and recomputed from its
predecessor's exit where that exit is not fresh, must give exactly the
oracle's whole-haystack find_iter (re_trait.rs:197-221) — for the chunked
kernels and for the wave-per-haystack path (assertions, Unicode \\b)."""
import numpy as np
import pytest

import regex_amd as R
from golden_data import corpus, known_counts
from oracle_py import OracleRegex
from regex_amd.dist import find_iter_spans_local, span_bounds

pytestmark = pytest.mark.gpu

CHUNK = [r"\w+", r"a+", r"x*", r"(?s).", r">[^\n]*\n|\n", r"\n", r'"[^"]*"', r"[a-q][^u-z]{13}x", r"agggtaaa|tttaccct", r""]
WAVE = [r"\b\w+\b", r"(?m)^\w+$", r"\bthe\b", r"\B"]


def dev(buf, cuda):
    import torch
    t = torch.zeros(len(buf) + 16, dtype=torch.uint8)
    t[: len(buf)] = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy())
    return t.to(cuda)


def pairs(m):
    return [(int(a), int(b)) for a, b in m.cpu().numpy()]


@pytest.mark.parametrize("pat", CHUNK + WAVE)
@pytest.mark.parametrize("k", [1, 2, 3, 8])
def test_spans_sherlock(cuda, pat, k):
    text = corpus("sherlock")[:150000]
    re = R.Regex(pat)
    exp = OracleRegex(re).find_iter(text)
    got, _ = find_iter_spans_local(re, dev(text, cuda), len(text), k)
    assert pairs(got) == exp


@pytest.mark.parametrize("pat", [r"a+", r"a*", r"(a|ab)(c|bcd)(d*)", r"\w+\s+\w+"])
def test_spans_cross_every_cut(cuda, pat):
    # long runs put a match across every cut: the exit exchange must recompute
    text = (b"b" + b"a" * 997 + b"cd ") * 40
    re = R.Regex(pat)
    exp = OracleRegex(re).find_iter(text)
    for k in (2, 5, 16, 64):
        got, rounds = find_iter_spans_local(re, dev(text, cuda), len(text), k)
        assert pairs(got) == exp, k


def test_span_exit_fresh_and_entry(cuda):
    # one span's exit fed by hand into the next (the C ABI contract)
    text = b"xx" + b"a" * 100 + b"yy"
    re = R.Regex(r"a+")
    h = dev(text, cuda)
    c0, m0, ex0 = re.find_iter_span(h, 0, 50, length=len(text))
    assert pairs(m0) == [(2, 102)]
    e = ex0.tolist()
    assert e[2] == 0 and e[0] == 102   # the match runs past the cut: not fresh
    c1, m1, ex1 = re.find_iter_span(h, 50, len(text), length=len(text), entry=ex0)
    assert pairs(m1) == []
    c1f, m1f, _ = re.find_iter_span(h, 50, len(text), length=len(text))
    assert pairs(m1f) == [(50, 102)]  # the speculative result the exchange corrects


def test_spans_regexdna_known_answers(cuda):
    kc = known_counts()["regexdna"]
    raw = corpus("regexdna")
    text = raw * 3
    strip = R.Regex(kc["strip"])
    exp = OracleRegex(strip).find_iter(text)
    got, _ = find_iter_spans_local(strip, dev(text, cuda), len(text), 7)
    assert pairs(got) == exp
    seq = R.Regex(kc["strip"]).replace_all(raw, b"")
    assert len(seq) == kc["stripped_len"]
    for v in kc["variants"]:
        re = R.Regex(v["re"])
        got, _ = find_iter_spans_local(re, dev(seq, cuda), len(seq), 5)
        assert len(pairs(got)) == v["count"], v["re"]


def _chain(re, h, n, bounds):
    """iterate_spans over arbitrary span bounds [b0, b1), [b1, b2), ..."""
    import torch
    from regex_amd.dist import iterate_spans
    k = len(bounds) - 1

    def run(i, entry):
        ent = None if entry is None else torch.tensor(entry, dtype=torch.int64, device=h.device)
        return re.find_iter_span(h, bounds[i], bounds[i + 1], length=n, entry=ent)

    res, rounds = iterate_spans(run, k, list(range(k)), lambda mine: [mine[i].tolist() for i in range(k)])
    return [m for i in range(k) for m in pairs(res[i][1])], rounds


@pytest.mark.parametrize("pat", [r"a+", r"a*", r"\ba+\b", r"(?m)^a+$", r"x|a{3}"])
def test_spans_custom_bounds(cuda, pat):
    # empty spans, spans inside one long match, a span starting mid-match,
    # spans of one byte, and the empty-match rule at every cut
    text = b"x" + b"a" * 300 + b"y\naaa\n" + b"ab" * 40 + b"a" * 5
    n = len(text)
    re = R.Regex(pat)
    exp = OracleRegex(re).find_iter(text)
    h = dev(text, cuda)
    for bounds in ([0, 5, 5, 100, 200, 302, n], [0, 1, 2, 3, 301, 302, 303, n], [0, 0, n], [0, n, n],
                   list(range(0, n, 7)) + [n]):
        got, _ = _chain(re, h, n, bounds)
        assert got == exp, (pat, bounds)


def test_span_entry_past_the_span(cuda):
    # a match that covers a whole span: that span owns nothing and passes the
    # entry on unchanged (not fresh)
    text = b"x" + b"a" * 300 + b"y"
    re = R.Regex(r"a+")
    h = dev(text, cuda)
    c0, m0, e0 = re.find_iter_span(h, 0, 10, length=len(text))
    assert pairs(m0) == [(1, 301)]
    c1, m1, e1 = re.find_iter_span(h, 10, 20, length=len(text), entry=e0)
    assert pairs(m1) == [] and e1.tolist() == e0.tolist()
