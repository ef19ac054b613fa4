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


def max_over_ranks(seconds, device, group=None):
    """The slowest rank's time (the bench contract: max over ranks)."""
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
