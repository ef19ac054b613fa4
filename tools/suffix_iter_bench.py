"""find_iter of DfaSuffix regexes over one long haystack (~1 GiB of sherlock
text): the parallel suffix iteration (launch_suffix_iter) against the wave
path it replaces (knob suffix_iter=0: lane 0 of one wave walks the
haystack), the latter on a 16 MiB prefix; outputs compared on the prefix.
usage: python tools/suffix_iter_bench.py"""
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
copies = (1 << 30) // len(raw)
L = len(raw) * copies
buf = torch.zeros(L + 16, dtype=torch.uint8, device=dev)
one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
buf[:L].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))
P = 16 << 20


def run(re, n, cap):
    return re.find_iter_batch(buf, stride=n, length=n, count=1, capacity=cap)


for pat in (r"[a-z]+ing", r"\w+@gmail\.com", r"\w+\s+Holmes"):
    re = R.Regex(pat)
    c, m = run(re, L, 1)
    total = int(c[0].item())
    cap = max(total, 1)
    run(re, L, cap)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        c, m = run(re, L, cap)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    path = N.rure_amd_last_fwd_path()
    cp, mp = run(re, P, cap)
    fast = mp.cpu().numpy()
    R._debug_set("suffix_iter=%s" % ("0"))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cw, mw = run(re, P, cap)
    torch.cuda.synchronize()
    wave_ms = (time.perf_counter() - t0) * 1e3
    R._debug_set(None)
    print(json.dumps({"pattern": pat, "match_type": re.match_info()["match_type"], "bytes": L, "matches": total,
                      "iter_ms": round(ms, 3), "iter_GBps": round(L / ms / 1e6, 1), "path": path,
                      "wave_ms_16MiB": round(wave_ms, 1), "wave_GBps": round(P / wave_ms / 1e6, 3),
                      "prefix_outputs_equal": bool(np.array_equal(fast, mw.cpu().numpy()))}), flush=True)
