"""World-size-2 gloo tests (CPU) of the multi-GPU plumbing (regex_amd/dist.py):
sharding covers every haystack exactly once, and the record gather returns
every rank's matches in rank order with global haystack ids — the exchange
step bench.py runs over RCCL for N > 1."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from regex_amd.dist import compact_matches, gather_records, max_over_ranks, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_total = 1001
        lo, hi = shard_range(n_total, world, rank)
        # synthetic per-haystack find results: a match in every 7th haystack
        idx = torch.arange(lo, hi)
        found = torch.full((hi - lo, 2), -1, dtype=torch.int64)
        m = idx % 7 == 0
        found[m, 0] = idx[m] * 3
        found[m, 1] = idx[m] * 3 + 10
        rec = compact_matches(found, lo)
        allrec = gather_records(rec)
        t = max_over_ranks(0.5 + rank, torch.device("cpu"))
        q.put((rank, lo, hi, allrec.tolist(), t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_records_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # shards tile [0, n) exactly
    assert res[0][1] == 0 and res[-1][2] == 1001
    for a, b in zip(res, res[1:]):
        assert a[2] == b[1]
    exp = [[i, 3 * i, 3 * i + 10] for i in range(1001) if i % 7 == 0]
    for r in res:
        assert r[3] == exp        # every rank sees all records, in rank order
        assert r[4] == 0.5 + (world - 1)


def test_shard_range_covers():
    for n in (0, 1, 5, 1000):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1


# ----------------------------------------------- sharded find_iter protocol
# The exit exchange of regex_amd.dist.iterate_spans, run over gloo with the
# CPU oracle as each rank's span iteration (the GPU runs the same protocol
# through rure_amd_find_iter_span, tests/test_gpu_span.py).  The oracle span
# reports "fresh" only for the literal fresh state, so every match crossing a
# cut forces a recomputation round.

SPAN_CASES = [
    (r"a+", b"xx" + b"a" * 40 + b"yy" + b"a" * 7 + b"z" * 5 + b"a" * 30),
    (r"a*", b"baab" * 9 + b"aaaa" * 10),
    (r">[^\n]*\n|\n", b">ONE Homo sapiens alu\nGGCCGGGCGCGG\n>TWO IUB ambiguity\nacgt\n" * 3),
    (r"agggtaaa|tttaccct", b"cagggtaaattttaccctgg" * 5),
    (r"", b"abcdef"),
    (r"(?m)^\w+$", b"foo\nbar baz\nqux\n\nlast"),
]


def _oracle_span(o, text, lo, hi, entry):
    """The span iteration of rure_amd_find_iter_span on the CPU oracle."""
    last = hi == len(text)
    if entry is None:
        p, lm = lo, None
    else:
        p, lm = int(entry[0]), (None if int(entry[1]) < 0 else int(entry[1]))
    out = []
    while p <= len(text):
        m = o.find(text, p)
        if m is None:
            break
        s, e = m
        if not last and s >= hi:
            break
        if s == e:
            p = e + 1
            if lm == e:
                continue
        else:
            p = e
        lm = e
        out.append((s, e))
    ex = [p, -1 if lm is None else lm, 1 if (p == hi and lm != hi) else 0]
    return len(out), out, torch.tensor(ex, dtype=torch.int64)


def _span_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import regex_amd as R
        from oracle_py import OracleRegex
        from regex_amd.dist import iterate_spans, span_bounds
        got = []
        for pat, text in SPAN_CASES:
            o = OracleRegex(R.Regex(pat))

            def run(i, entry):
                lo, hi = span_bounds(len(text), world, i)
                return _oracle_span(o, text, lo, hi, entry)

            def gather(mine):
                parts = [torch.empty(3, dtype=torch.int64) for _ in range(world)]
                dist.all_gather(parts, mine[rank])
                return [p.tolist() for p in parts]

            res, rounds = iterate_spans(run, world, [rank], gather)
            parts = [None] * world
            dist.all_gather_object(parts, res[rank][1])
            got.append(([m for p in parts for m in p], rounds, o.find_iter(text)))
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_find_iter_sharded_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_span_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    crossed = 0
    for _, got in res:
        for (pat, _), (merged, rounds, exp) in zip(SPAN_CASES, got):
            assert merged == exp, pat
            crossed += rounds
    assert crossed > 0   # some cases cross a cut and exercise the repair rounds


def test_iterate_spans_single_process():
    """Every span count on one process (the find_iter_spans_local shape)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import regex_amd as R
    from oracle_py import OracleRegex
    from regex_amd.dist import iterate_spans, span_bounds
    for pat, text in SPAN_CASES:
        o = OracleRegex(R.Regex(pat))
        exp = o.find_iter(text)
        for k in (1, 2, 3, 5, 8, len(text) + 1):
            def run(i, entry):
                lo, hi = span_bounds(len(text), k, i)
                return _oracle_span(o, text, lo, hi, entry)
            res, _ = iterate_spans(run, k, list(range(k)), lambda mine: [mine[i].tolist() for i in range(k)])
            assert [m for i in range(k) for m in res[i][1]] == exp, (pat, k)
