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
