"""Throughput of the one-wave-per-haystack find_iter path (iter_wave_kernel:
DFA on lane 0, Pike VM on the wave after a quit) with many haystacks in
flight: a Unicode-\\b regex over copies of sherlock as it is (non-ASCII
bytes quit its DFA), one copy per haystack.  The rate a chunked version
would reach with units in place of haystacks."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch

import regex_amd as R
from regex_amd import _native as N
from golden_data import corpus

dev = torch.device("cuda", 0)
raw = corpus("sherlock")
for pat in sys.argv[1:] or [r"\b\w+n\b"]:
    re = R.Regex(pat)
    for L, count in ((16384, 4096), (65536, 1024), (len(raw) // 16 * 16, 64)):
        t = (raw * (L * count // len(raw) + 1))[:L * count]
        d = torch.from_numpy(np.frombuffer(t + bytes(16), dtype=np.uint8).copy()).to(dev)
        c, m = re.find_iter_batch(d, stride=L, length=L, count=count)
        path = N.rure_amd_last_fwd_path()
        cap = int(c.sum().item()) + 16
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            re.find_iter_batch(d, stride=L, length=L, count=count, capacity=cap)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 2 * 1e3
        print(json.dumps({"pattern": pat, "L": L, "count": count, "bytes": L * count, "ms": round(ms, 2),
                          "GBps": round(L * count / ms / 1e6, 3), "matches": cap - 16, "path": path}), flush=True)
