"""replacen on the regex-dna stream (rure_amd_replace_batch): kernel-level
timing of the strip (35 M deletions) and one IUB substitution, with a fresh
output buffer per call (as regex_amd/shootout.py allocates) and with one
reused buffer; plus a plain fill of a fresh vs a reused buffer of the same
size (first-touch cost of freshly allocated device memory)."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import regex_amd as R  # noqa: E402
from regex_amd import _native as N  # noqa: E402
from golden_data import corpus  # noqa: E402


def ms(fn, reps=3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    raw = corpus("regexdna")
    copies = (1 << 31) // len(raw)
    n = copies * len(raw)
    one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
    big = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    big[:n].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))
    big[n:] = 0
    ooff = torch.empty((2,), dtype=torch.int64, device=dev)
    total = torch.zeros((1,), dtype=torch.int64, device=dev)

    def rep(re_, buf, ln, r, out):
        b = N.RureBatch()
        b.haystack = buf.data_ptr(); b.offsets = None; b.stride = ln; b.length = ln; b.count = 1; b.start = 0
        rc = N.rure_amd_replace_batch(re_._re, ctypes.byref(b), r, len(r), 0, ctypes.c_void_p(out.data_ptr()),
                                      ctypes.c_void_p(ooff.data_ptr()), out.numel() - 16,
                                      ctypes.c_void_p(total.data_ptr()), None)
        assert rc == 0

    strip = R.Regex(rb">[^\n]*\n|\n")
    cap = n + n // 4
    out = torch.empty(cap + 16, dtype=torch.uint8, device=dev)
    rep(strip, big, n, b"", out)
    torch.cuda.synchronize()
    cl = int(total.item())
    print("strip reused out: %.2f ms" % ms(lambda: rep(strip, big, n, b"", out)), flush=True)
    print("strip fresh out: %.2f ms" % ms(lambda: rep(strip, big, n, b"",
                                                     torch.empty(cap + 16 + int(time.time_ns() % 4096),
                                                                 dtype=torch.uint8, device=dev))), flush=True)
    stripped = out[:cl + 16].clone()
    sub = R.Regex(b"B")
    out2 = torch.empty(cl + cl // 4 + 16, dtype=torch.uint8, device=dev)
    print("IUB B reused out: %.2f ms" % ms(lambda: rep(sub, stripped, cl, b"(c|g|t)", out2)), flush=True)
    x = torch.empty(cap, dtype=torch.uint8, device=dev)
    print("fill reused: %.2f ms" % ms(lambda: x.fill_(1)), flush=True)
    print("fill fresh: %.2f ms" % ms(lambda: torch.empty(cap + int(time.time_ns() % 4096), dtype=torch.uint8,
                                                        device=dev).fill_(1)), flush=True)


if __name__ == "__main__":
    main()
