"""DfaAnchoredReverse byte reduction: find of the end-anchored date regex
`\\d{4}-\\d{2}-\\d{2}$` over the C2 batch (1M x 4 KiB, 1 % of the haystacks
end in a date) against the unanchored C2 find on the same batch.  Prints the
kernel times (HIP events) and the oracle's forward / reverse byte counts on a
sample (the reference's own work).  python tools/anchored_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch

import regex_amd as R
from oracle_py import OracleRegex
from regex_amd.workloads import date_haystacks_device

dev = torch.device("cuda", 0)
n, L = 1 << 20, 4096
hay, planted = date_haystacks_device(n, L, 0x5EED0002, dev, frac=0.0)
idx = torch.arange(0, n, 100, device=dev)
date = torch.frombuffer(bytearray(b"2017-12-30"), dtype=torch.uint8).to(dev)
pos = (idx * L + (L - 10))[:, None] + torch.arange(10, device=dev)[None, :]
hay[pos.reshape(-1)] = date.repeat(idx.numel())
st = torch.cuda.current_stream(dev)
out = torch.empty((n, 2), dtype=torch.int64, device=dev)


def timed(re, reps=20):
    for _ in range(3):
        re.find_batch(hay, stride=L, length=L, count=n, out=out, stream=st)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        re.find_batch(hay, stride=L, length=L, count=n, out=out, stream=st)
        b.record(st)
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))


res = {}
for pat in (r"\d{4}-\d{2}-\d{2}$", r"\d{4}-\d{2}-\d{2}"):
    re = R.Regex(pat)
    ms = timed(re)
    got = out.cpu().numpy()
    S = 8192
    o = OracleRegex(re)
    buf = hay[: S * L].cpu().numpy()
    exp, stt = o.find_batch(buf, L, L, S, nthreads=8)
    assert np.array_equal(got[:S], exp.astype(np.int64)), pat
    res[pat] = {"kernel_ms": round(ms, 4), "matched": int((got[:, 0] >= 0).sum()),
                "oracle_fwd_bytes_per_haystack": stt["fwd_bytes"] / S, "oracle_rev_bytes_per_haystack": stt["rev_bytes"] / S,
                "logical_GBps": round(n * L / ms / 1e6, 1)}
import json
print(json.dumps(res))
