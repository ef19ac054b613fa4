"""find_iter of C+ regexes (the run engine, run_iter.hip, last_fwd_path
-19) over 1 GiB of sherlock text (as it is, with its non-ASCII bytes; or
made ASCII with --ascii), against the DFA paths (knob runs=0: the ASCII
shadow / chunked iteration); outputs of the two compared in full (count and
every record).  One JSON line per pattern.
usage: python tools/runs_bench.py [--ascii] [pattern ...]"""
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
ascii_only = "--ascii" in sys.argv
argv = [a for a in sys.argv[1:] if a != "--ascii"]
raw = corpus("sherlock")
if ascii_only:
    raw = bytes(b if b < 0x80 else 0x20 for b in raw)
copies = (1 << 30) // len(raw)
L = len(raw) * copies
buf = torch.zeros(L + 16, dtype=torch.uint8, device=dev)
one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
buf[:L].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))


def run(re, reps):
    c, m = re.find_iter_batch(buf, stride=L, length=L, count=1, capacity=1)
    cap = max(int(c[0].item()), 1)
    c, m = re.find_iter_batch(buf, stride=L, length=L, count=1, capacity=cap)
    path = N.rure_amd_last_fwd_path()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        re.find_iter_batch(buf, stride=L, length=L, count=1, capacity=cap)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, int(c[0].item()), m, path


pats = argv or [r"\w+", r"[a-z]+", r"\S+", r"\pL+", r"\d+", r"[^\n]+"]
for pat in pats:
    R._debug_set(None)
    ms, n, m, path = run(R.Regex(pat), 5)
    R._debug_set("runs=%s" % ("0"))
    ms0, n0, m0, path0 = run(R.Regex(pat), 2)
    R._debug_set(None)
    same = n == n0 and bool(torch.equal(m, m0))
    alg = L + 16 * n
    print(json.dumps({"pattern": pat, "text": "sherlock ascii" if ascii_only else "sherlock", "bytes": L, "matches": n, "runs_ms": round(ms, 3), "runs_path": path,
                      "runs_GBps": round(L / ms / 1e6, 1), "alg_bytes": alg,
                      "runs_alg_TBps": round(alg / ms / 1e9, 3), "dfa_ms": round(ms0, 3), "dfa_path": path0,
                      "speedup": round(ms0 / ms, 2), "outputs_equal": same}), flush=True)
