"""C4 set kernel variants in one process: the 10 M-line C4 batch timed under
several debug-knob settings (HIP events, 20 calls each, 3 alternating
passes), outputs compared with the default's.  One JSON line per setting.
usage: python tools/c4_ab.py "core_order=0" "core_early=1" ..."""
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
settings = [""] + sys.argv[1:]
ref = torch.empty(n, dtype=torch.int64, device=dev)
R._debug_set(None)
rs.matches_batch(buf, offsets=offs, out=ref)
best = {}
for rnd in range(3):
    for st in settings:
        R._debug_set(st or None)
        out = torch.empty(n, dtype=torch.int64, device=dev)
        t = timed(lambda: rs.matches_batch(buf, offsets=offs, out=out))
        ok = bool(torch.equal(out, ref))
        b = best.setdefault(st, [1e9, True])
        b[0] = min(b[0], t)
        b[1] = b[1] and ok
R._debug_set(None)
nb = int(offs[-1].item())
for st in settings:
    print(json.dumps({"tool": "tools/c4_ab.py", "knobs": st or "default", "ms": round(best[st][0], 4),
                      "GBps": round(nb / best[st][0] / 1e6, 1), "outputs_equal": best[st][1]}), flush=True)
