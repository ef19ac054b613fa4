"""Batched find over a >65535-state automaton: the big-DFA kernel
(big_dfa.hip) against the Pike VM (knob big=0), GB/s.
python tools/big_dfa_bench.py [pattern] [count] [length]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch

import regex_amd as R
from regex_amd import _native as N

pat = sys.argv[1] if len(sys.argv) > 1 else r"[a-q][^u-z]{13}x"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
L = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
dev = torch.device("cuda:0")
rng = np.random.default_rng(1)
buf = torch.from_numpy(rng.choice(np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", dtype=np.uint8), size=n * L + 16)).to(dev)
t0 = time.time()
re = R.Regex(pat)
info = re.dfa_info(3)
print("compile+build %.2f s" % (time.time() - t0), info, flush=True)
out = torch.empty((n, 2), dtype=torch.int64, device=dev)
res = {}
for mode in ("2", "0"):
    R._debug_set("big=%s" % (mode))
    re.find_batch(buf, stride=L, length=L, count=n, out=out)
    torch.cuda.synchronize()
    reps = 3 if mode == "2" else 1
    t = time.time()
    for _ in range(reps):
        re.find_batch(buf, stride=L, length=L, count=n, out=out)
    torch.cuda.synchronize()
    dt = (time.time() - t) / reps
    res[mode] = out.cpu().numpy().copy()
    print("%s: %.3f ms  %.1f GB/s  path %d  matches %d" % ("big DFA" if mode == "2" else "Pike VM", dt * 1e3,
          n * L / dt / 1e9, N.rure_amd_last_fwd_path(), int((res[mode][:, 0] >= 0).sum())), flush=True)
print("agree", bool((res["2"] == res["0"]).all()))
