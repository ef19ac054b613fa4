"""find_iter of regexes that take the ASCII shadow automaton (DESIGN §4.3:
by default the shadow's quit is a device flag gating both passes, path -25;
with knob shadow_sync=1 it is read back, -14 = the shadow answered, -15 = a
unit quit on a non-ASCII byte and the batch re-ran on the full automaton)
against the full automaton alone (knob ascii_shadow=0), over 1 GiB of sherlock text three ways: made
ASCII, as it is (sparse non-ASCII bytes), and dense (every 64th byte's word
turned into a two-byte UTF-8 letter).  Outputs of the two compared in full.
One JSON line per pattern and text.  (Not a Unicode-\b regex by default: on
text with non-ASCII bytes its DFA quits for good and the batch goes to the
one-wave-per-haystack path, minutes for one 1 GiB haystack — as the
reference's lazy DFA hands such a search to its NFA engines.)
usage: python tools/shadow_bench.py [pattern ...]"""
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


def texts():
    yield "ascii", bytes(b if b < 0x80 else 0x20 for b in raw0)
    yield "as_is", raw0
    a = bytearray(raw0)
    for i in range(0, len(a) - 1, 64):  # a letter pair -> U+00E9 (0xC3 0xA9)
        if 0x61 <= a[i] <= 0x7A and 0x61 <= a[i + 1] <= 0x7A:
            a[i], a[i + 1] = 0xC3, 0xA9
    yield "dense", bytes(a)


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


pats = sys.argv[1:] or [r"\w+\s+\w+", r"(?m)^\w+"]
for name, raw in texts():
    buf, L = device_text(raw)
    for pat in pats:
        R._debug_set(None)
        ms, n, m, path = run(R.Regex(pat), buf, L, 3)
        R._debug_set("shadow_sync=1")
        ms1, n1, m1, path1 = run(R.Regex(pat), buf, L, 3)
        R._debug_set("ascii_shadow=0")
        ms0, n0, m0, path0 = run(R.Regex(pat), buf, L, 3)
        R._debug_set(None)
        print(json.dumps({"pattern": pat, "text": name, "bytes": L, "matches": n, "shadow_ms": round(ms, 3),
                          "shadow_path": path, "sync_ms": round(ms1, 3), "sync_path": path1,
                          "sync_equal": n == n1 and bool(torch.equal(m, m1)),
                          "full_ms": round(ms0, 3), "full_path": path0,
                          "shadow_speedup": round(ms0 / ms, 2), "outputs_equal": n == n0 and bool(torch.equal(m, m0))}),
              flush=True)
    del buf
