"""The wave-served chunked find_iter (last_fwd_path -27) over 1 GiB of
sherlock: as it is (33 non-ASCII bytes per 594 KB copy quit the DFA of a
Unicode \\b) and made ASCII; on ASCII text also with knob iter_wave=0 (the
plain chunked iteration that reads its quit flag back, -12), the cost of
the wave mode where nothing quits.  One JSON line per pattern and text.
usage: python tools/wave_iter_bench.py [pattern ...]"""
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
raw0 = corpus("sherlock")


def device_text(raw):
    copies = (1 << 30) // len(raw)
    L = len(raw) * copies
    buf = torch.zeros(L + 16, dtype=torch.uint8, device=dev)
    one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
    buf[:L].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))
    return buf, L


def run(re, buf, L, reps):
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


pats = sys.argv[1:] or [r"\b\w+n\b", r"\b\w+\b"]
KN = os.environ.get("WAVE_KNOBS") or None  # a debug spec for the default runs (A/B of unit sizes)
TEXTS = os.environ.get("WAVE_TEXTS", "as_is,ascii").split(",")
for name, raw in (("as_is", raw0), ("ascii", bytes(b if b < 0x80 else 0x20 for b in raw0))):
    if name not in TEXTS:
        continue
    buf, L = device_text(raw)
    for pat in pats:
        R._debug_set(KN)
        ms, n, m, path = run(R.Regex(pat), buf, L, 3)
        R._debug_set(None)
        line = {"pattern": pat, "text": name, "bytes": L, "matches": n, "ms": round(ms, 3), "path": path,
                "GBps": round(L / ms / 1e6, 2), "knobs": KN}
        if name == "ascii":
            R._debug_set("iter_wave=0")
            ms0, n0, m0, path0 = run(R.Regex(pat), buf, L, 3)
            R._debug_set(None)
            line.update({"plain_ms": round(ms0, 3), "plain_path": path0,
                         "outputs_equal": n == n0 and bool(torch.equal(m, m0))})
        print(json.dumps(line), flush=True)
    del buf
