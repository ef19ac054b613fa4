"""Multi-GPU plumbing for the batched scan.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on
ROCm).  The scan itself never communicates: every rank owns an independent
shard of haystacks (C2, C4) or one whole haystack (C5).  The only exchange is
gathering the match records, which these helpers do with a count exchange
followed by a padded all-gather (records are 3 x int64: global haystack id,
start, end).  They are backend-agnostic, so the same code is tested on CPU
with gloo (tests/test_dist.py).
"""
import torch
import torch.distributed as dist


def shard_range(n, world, rank):
    """Contiguous [lo, hi) slice of n units for `rank` (sizes differ by <= 1)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def compact_matches(found, base):
    """(k, 3) records (base + haystack index, start, end) of the haystacks
    whose find result (n, 2) holds a match (start >= 0)."""
    hit = (found[:, 0] >= 0).nonzero().squeeze(1)
    rec = torch.empty((hit.numel(), 3), dtype=torch.int64, device=found.device)
    rec[:, 0] = hit + base
    rec[:, 1:] = found[hit]
    return rec


def gather_records(rec, group=None):
    """All-gather variable-length (k_r, 3) int64 record tensors; returns the
    concatenation in rank order on every rank."""
    world = dist.get_world_size(group)
    k = torch.tensor([rec.shape[0]], dtype=torch.int64, device=rec.device)
    ks = [torch.zeros_like(k) for _ in range(world)]
    dist.all_gather(ks, k, group=group)
    kmax = max(int(x.item()) for x in ks)
    pad = torch.full((max(kmax, 1), 3), -1, dtype=torch.int64, device=rec.device)
    pad[: rec.shape[0]] = rec
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[: int(c.item())] for p, c in zip(parts, ks)], dim=0)


def _all_gather_flat(out, inp, group=None):
    """all_gather into one (world * rows, ...) tensor (no per-part copies);
    backends without the flat collective get the list form."""
    if not dist.is_initialized():  # one process, no group: the gather is a copy
        out.copy_(inp)
        return
    try:
        dist.all_gather_into_tensor(out, inp, group=group)
    except (RuntimeError, NotImplementedError, AttributeError):
        dist.all_gather(list(out.chunk(dist.get_world_size(group))), inp, group=group)


class RecordGather(object):
    """Sync-free gathering of a rank's find results (the path's
    only exchange).  Every step: the device compacts the (n, 2) find output
    into (base + haystack, start, end) records with their count
    (rure_amd_compact_matches, one HIP kernel pair, no host round trip), then
    one all-gather of a fixed-capacity (capacity + 1, 3) block per rank — row
    0 holds the count.  Nothing is read back until result(), after the timed
    region, which also detects a capacity overflow."""

    def __init__(self, capacity, device, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.cap = int(capacity)
        self.send = torch.zeros((self.cap + 1, 3), dtype=torch.int64, device=device)
        self.recv = torch.empty((self.world * (self.cap + 1), 3), dtype=torch.int64, device=device)

    def compact(self, found, base, stream=None):
        import ctypes
        from . import _native as N, _stream_ptr
        rc = N.rure_amd_compact_matches(ctypes.c_void_p(found.data_ptr()), found.shape[0], int(base),
                                        ctypes.c_void_p(self.send[1:].data_ptr()), self.cap,
                                        ctypes.c_void_p(self.send.data_ptr()), _stream_ptr(stream))
        if rc != N.OK:
            raise RuntimeError("rure_amd_compact_matches failed (%d)" % rc)

    def step(self, found, base, stream=None):
        if found.is_cuda:
            self.compact(found, base, stream)
            # the collective runs on torch's current stream: order it after
            # the compaction when that ran on another stream
            if stream is not None and stream != torch.cuda.current_stream(found.device):
                torch.cuda.current_stream(found.device).wait_stream(stream)
        else:  # CPU rehearsal (gloo tests): the same layout from torch ops
            rec = compact_matches(found, base)
            k = rec.shape[0]
            self.send[0, 0] = k
            self.send[1:1 + min(k, self.cap)] = rec[: self.cap]
        _all_gather_flat(self.recv, self.send, self.group)

    def result(self):
        """(records of every rank in rank order, per-rank counts); raises
        OverflowError if a rank found more matches than the capacity."""
        blocks = self.recv.view(self.world, self.cap + 1, 3)
        counts = blocks[:, 0, 0].tolist()
        if max(counts) > self.cap:
            raise OverflowError("match records exceed the gather capacity (%d > %d)" % (max(counts), self.cap))
        return torch.cat([blocks[r, 1:1 + c] for r, c in enumerate(counts)], dim=0), counts


def max_over_ranks(seconds, device, group=None):
    """The slowest rank's time (the bench contract: max over ranks)."""
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


# ----------------------------------------------------- sharded find_iter (C3)
# One logical haystack (regex-dna's 2 GiB stream) cut into contiguous spans,
# one per rank.  Every rank iterates its span speculatively from a fresh start
# (rure_amd_find_iter_span); the exits are exchanged (an all-gather of 3 x
# int64 per rank) and a rank whose predecessor's exit is not equivalent to a
# fresh start recomputes its span entered with that exit.  Rank r's exit is
# final once ranks < r are, so this takes at most world - 1 rounds; with no
# match crossing a cut it takes none.


def _entry_key(ex):
    ex = [int(x) for x in ex]
    return ("fresh",) if ex[2] else (ex[0], ex[1])


def iterate_spans(run_span, nspans, mine, gather_exits):
    """Exact chained iteration over `nspans` spans.

    run_span(i, entry) -> (count, matches, exit) runs span i entered with
    `entry` (None = fresh, else (next, last_match, 0)); exit is a 3-int
    sequence or tensor (next, last_match, fresh).  `mine` = the span ids this
    process runs; gather_exits({i: exit}) -> list of every span's exit.
    Returns ({i: result}, rounds of recomputation)."""
    res = {i: run_span(i, None) for i in mine}
    used = [("fresh",)] * nspans
    rounds = 0
    while True:
        exits = gather_exits({i: res[i][2] for i in mine})
        redo = [i for i in range(1, nspans) if _entry_key(exits[i - 1]) != used[i]]
        if not redo:
            return res, rounds
        rounds += 1
        for i in redo:
            used[i] = _entry_key(exits[i - 1])
            if i in res:
                k = used[i]
                res[i] = run_span(i, None if k == ("fresh",) else (k[0], k[1], 0))


def span_bounds(length, nspans, i):
    """[lo, hi) of span i; the last span ends at `length` (and owns an empty
    match at the very end)."""
    return shard_range(length, nspans, i)


def find_iter_sharded(re, hay, length, group=None, stream=None):
    """bytes::Regex::find_iter over one haystack sharded across the ranks of
    `group` (every rank holds the haystack; each scans its own span).
    Returns (matches owned by this rank, global index of its first match,
    total matches, recomputation rounds)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)

    def run(i, entry):
        lo, hi = span_bounds(length, world, i)
        ent = None if entry is None else torch.tensor(entry, dtype=torch.int64, device=hay.device)
        return re.find_iter_span(hay, lo, hi, length=length, entry=ent, stream=stream)

    def gather(mine):
        ex = mine[rank]
        parts = [torch.empty_like(ex) for _ in range(world)]
        dist.all_gather(parts, ex, group=group)
        return [p.tolist() for p in parts]

    res, rounds = iterate_spans(run, world, [rank], gather)
    count, matches, _ = res[rank]
    counts = [torch.empty_like(count) for _ in range(world)]
    dist.all_gather(counts, count, group=group)
    counts = [int(c.item()) for c in counts]
    return matches, sum(counts[:rank]), sum(counts), rounds


def find_iter_spans_local(re, hay, length, nspans, stream=None):
    """The same chained span iteration with every span on this device (tests
    and single-GPU rehearsal of the sharded protocol).  Returns (matches in
    order, rounds)."""
    def run(i, entry):
        lo, hi = span_bounds(length, nspans, i)
        ent = None if entry is None else torch.tensor(entry, dtype=torch.int64, device=hay.device)
        return re.find_iter_span(hay, lo, hi, length=length, entry=ent, stream=stream)

    res, rounds = iterate_spans(run, nspans, list(range(nspans)),
                                lambda mine: [mine[i].tolist() for i in range(nspans)])
    return torch.cat([res[i][1] for i in range(nspans)], dim=0), rounds
