"""The on-demand DFA (debug knob lazy, host LazyDfa + lazy_dfa_kernel) on a
regex past the eager budgets, `(?:a|b)*a(?:a|b){20}`, over a batch of
sherlock lines mixed with a/b runs: first call (the eager attempt that
fails, then the rounds that build the rows the text needs) and steady state
(every row the text visits built: one round), against the Pike VM
(lazy=0; its path is -16, the Pike VM alone).  Prints one JSON line per mode.
usage: python tools/lazy_bench.py [haystacks] [length] [sparse|dense]"""
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
L = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
pat = r"(?:a|b)*a(?:a|b){20}"
rng = np.random.default_rng(1)
base = corpus("sherlock")
# sherlock text with a/b runs planted: "dense" = a third of the pieces are
# random a/b runs of 1-40 bytes (millions of distinct 21-byte windows: every
# window is a DFA state, past the memory budget for find, as the reference's
# cache would thrash); "sparse" = 1 % of the pieces, runs of 22-30 bytes
text_kind = sys.argv[3] if len(sys.argv) > 3 else "sparse"
parts, total = [], 0
while total < n * L:
    if (text_kind == "dense" and rng.integers(0, 3) == 0) or (text_kind == "sparse" and rng.integers(0, 100) == 0):
        k = int(rng.integers(1, 40)) if text_kind == "dense" else int(rng.integers(22, 31))
        x = bytes(rng.choice(np.frombuffer(b"ab", dtype=np.uint8), size=k))
    else:
        a = int(rng.integers(0, len(base) - 100))
        x = base[a:a + int(rng.integers(1, 100))]
    parts.append(x)
    total += len(x)
raw = b"".join(parts)[:n * L]
dev = torch.device("cuda", 0)
d = torch.from_numpy(np.frombuffer(raw + b"\0" * 16, dtype=np.uint8).copy()).to(dev)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


# the default dispatch's first call: the eager big automaton is attempted
# first (kBigDfaRawStates) and fails, then the on-demand DFA runs
R._debug_set(None)
re0 = R.Regex(pat)
t0 = time.perf_counter()
re0.is_match_batch(d, stride=L, length=L, count=n)
torch.cuda.synchronize()
default_first = (time.perf_counter() - t0) * 1e3
default_path = N.rure_amd_last_fwd_path()
for mode in ("find", "is_match"):
    res = {}
    for lazy in ("1", "0"):
        # "1": forced on-demand DFA (no eager attempt first); "0": Pike VM
        # (the eager big automaton does not build: big=0 skips it)
        R._debug_set("lazy=%s,big=0" % lazy)
        re = R.Regex(pat)
        f = (lambda: re.find_batch(d, stride=L, length=L, count=n)) if mode == "find" else \
            (lambda: re.is_match_batch(d, stride=L, length=L, count=n))
        t0 = time.perf_counter()
        out = f()
        torch.cuda.synchronize()
        first = (time.perf_counter() - t0) * 1e3
        path = N.rure_amd_last_fwd_path()
        ms = timed(f, 5 if lazy == "1" else 1)
        res[lazy] = (first, ms, path, out.cpu().numpy())
    same = bool((res["1"][3] == res["0"][3]).all())
    print(json.dumps({"pattern": pat, "mode": mode, "text": text_kind, "haystacks": n, "length": L,
                      "lazy_first_call_ms": round(res["1"][0], 1), "lazy_ms": round(res["1"][1], 3),
                      "lazy_GBps": round(n * L / res["1"][1] / 1e6, 1), "lazy_path": res["1"][2],
                      "pike_ms": round(res["0"][1], 2), "pike_GBps": round(n * L / res["0"][1] / 1e6, 2),
                      "pike_path": res["0"][2], "outputs_equal": same,
                      "default_first_call_ms_is_match": round(default_first, 1), "default_path": default_path,
                      "matches": int((res["1"][3][:, 0] >= 0).sum() if mode == "find" else res["1"][3].sum())}),
          flush=True)
