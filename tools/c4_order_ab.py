"""How much of C4's set_core_kernel time is lane divergence over line
lengths: the C4 batch (10 M log lines, 64 patterns) as generated, and the
same lines reordered by length (a copy of the batch, lines sorted so that a
wave's 64 lines have nearly equal lengths), kernel time by HIP events.
Outputs compared (masks permuted back).  One JSON line.
usage: python tools/c4_order_ab.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import regex_amd as R  # noqa: E402
from regex_amd.workloads import C4_PATTERNS, log_lines_device  # noqa: E402


def timed(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


dev = torch.device("cuda:0")
n = 10_000_000
buf, offs = log_lines_device(n, dev, seed=0x5EED0004)
rs = R.RegexSet(C4_PATTERNS)
lens = offs[1:] - offs[:-1]
order = torch.argsort(lens, stable=True)
slen = lens[order]
soffs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
soffs[1:] = torch.cumsum(slen, 0)
total = int(soffs[-1].item())
# byte gather: for each output byte, its source (line start + offset in line)
line_of = torch.repeat_interleave(torch.arange(n, device=dev), slen)
pos = torch.arange(total, device=dev) - soffs[:-1][line_of]
src = offs[:-1][order][line_of] + pos
sbuf = torch.zeros(total + 16, dtype=torch.uint8, device=dev)
sbuf[:total] = buf[src]
del line_of, pos, src
out = torch.empty(n, dtype=torch.int64, device=dev)
sout = torch.empty(n, dtype=torch.int64, device=dev)
t0 = timed(lambda: rs.matches_batch(buf, offsets=offs, out=out))
t1 = timed(lambda: rs.matches_batch(sbuf, offsets=soffs, out=sout))
back = torch.empty_like(sout)
back[order] = sout
print(json.dumps({"lines": n, "bytes": total, "as_generated_ms": round(t0, 4), "sorted_by_length_ms": round(t1, 4),
                  "as_generated_GBps": round(total / t0 / 1e6, 1), "sorted_GBps": round(total / t1 / 1e6, 1),
                  "outputs_equal": bool(torch.equal(out, back))}), flush=True)
