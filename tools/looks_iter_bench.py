"""find_iter of look-around regexes over 1 GiB of sherlock text (made ASCII,
so Unicode \\b's DFA never quits): the chunked path (iter_scan.hip with
FwdDfaDev::looks, last_fwd_path -12) against the wave path
(knob iter_looks=0) on a 16 MiB prefix, outputs compared there.
--ragged: the same text as a ragged batch of its lines (one unit per line)
against the wave path, outputs compared.
usage: python tools/looks_iter_bench.py [--no-wave] [--ragged] [pattern ...]"""
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
raw = bytes(b if b < 0x80 else 0x20 for b in corpus("sherlock"))
copies = (1 << 30) // len(raw)
L = len(raw) * copies
buf = torch.zeros(L + 16, dtype=torch.uint8, device=dev)
one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
buf[:L].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))
SMALL = len(raw) * ((16 << 20) // len(raw))


def timed(re, n, reps):
    c, m = re.find_iter_batch(buf, stride=n, length=n, count=1, capacity=1)
    cap = max(int(c[0].item()), 1)
    re.find_iter_batch(buf, stride=n, length=n, count=1, capacity=cap)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        c, m = re.find_iter_batch(buf, stride=n, length=n, count=1, capacity=cap)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, cap, m


pats = [r"\b\w+\b", r"(?-u)\b\w+\b", r"\bthe\b", r"[a-z]+ed\b", r"(?m)^\w+", r"(?m)\w+$"]
args = [a for a in sys.argv[1:] if a not in ("--no-wave", "--ragged")]
wave = "--no-wave" not in sys.argv
if "--ragged" in sys.argv:
    small = bytes(raw) * 8  # ~4.7 MB of lines (the wave path is slow)
    ends = np.nonzero(np.frombuffer(small, dtype=np.uint8) == 10)[0] + 1
    offs = torch.from_numpy(np.concatenate([[0], ends]).astype(np.int64)).to(dev)
    hay = torch.from_numpy(np.frombuffer(small + b"\0" * 16, dtype=np.uint8).copy()).to(dev)

    def run(re):
        c, m = re.find_iter_batch(hay, offsets=offs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            c, m = re.find_iter_batch(hay, offsets=offs)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 3 * 1e3, m

    for pat in args or [r"\bthe\b", r"\b\w+\b", r"(?m)^\w+", r"[a-z]+ed\b"]:
        re = R.Regex(pat)
        ms, m = run(re)
        path = N.rure_amd_last_fwd_path()
        R._debug_set("iter_looks=%s" % ("0"))
        try:
            wms, wm = run(re)
        finally:
            R._debug_set(None)
        print(json.dumps({"pattern": pat, "ragged_lines": int(offs.numel() - 1), "bytes": len(small), "path": path,
                          "matches": int(m.shape[0]), "ms": round(ms, 3), "wave_ms": round(wms, 3),
                          "equal": bool(torch.equal(m, wm))}), flush=True)
    sys.exit(0)
for pat in args or pats:
    re = R.Regex(pat)
    ms, cap, _ = timed(re, L, 5)
    path = N.rure_amd_last_fwd_path()
    if not wave:
        print(json.dumps({"pattern": pat, "path": path, "matches": cap, "ms": round(ms, 3),
                          "GBps": round(L / ms / 1e6, 1)}), flush=True)
        continue
    _, _, m_small = timed(re, SMALL, 1)
    R._debug_set("iter_looks=%s" % ("0"))
    try:
        wms, wcap, m_wave = timed(re, SMALL, 1)
    finally:
        R._debug_set(None)
    same = bool(torch.equal(m_small, m_wave))
    print(json.dumps({"pattern": pat, "path": path, "matches": cap, "ms": round(ms, 3),
                      "GBps": round(L / ms / 1e6, 1), "wave_GBps_16MiB": round(SMALL / wms / 1e6, 3),
                      "equal_16MiB": same}), flush=True)
