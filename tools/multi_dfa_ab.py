"""Evidence for fusing general-DFA find_iter passes: each
regex's solo find_iter over ~1 GiB of sherlock text, its GB/s, its engine
and its DFA's LDS image size, against the HBM time of one read of the text.
A fused pass reads the text once but runs every regex's chain per byte and
needs every hot table in LDS at once.
usage: python tools/multi_dfa_ab.py"""
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
pats = [r"[A-Z][a-z]+\s+[A-Z][a-z]+", r"(?i)holmes\w*", r"\d+[a-z]*", r"Sherlock|Holmes", r"[a-z]+ing"]
total_ms = 0.0
for pat in pats:
    re = R.Regex(pat)
    c, m = re.find_iter_batch(buf, stride=L, length=L, count=1, capacity=1)
    cap = max(int(c[0].item()), 1)
    re.find_iter_batch(buf, stride=L, length=L, count=1, capacity=cap)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        re.find_iter_batch(buf, stride=L, length=L, count=1, capacity=cap)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 5 * 1e3
    total_ms += ms
    info = re.match_info()
    print(json.dumps({"pattern": pat, "match_type": info["match_type"], "path": N.rure_amd_last_fwd_path(),
                      "matches": cap, "ms": round(ms, 3), "GBps": round(L / ms / 1e6, 1)}), flush=True)
print(json.dumps({"sum_of_solo_ms": round(total_ms, 3), "one_read_at_6TBps_ms": round(L / 6e9, 3),
                  "bytes": L}), flush=True)
