"""A/B of the start-state prefix skip (dfa.rs:700-711) on the chunked long
scan (long_scan_kernel, last_fwd_path -4) over ~1 GiB of sherlock text as one
haystack: no skip (debug knob prefix=0), the first-byte skip (prefix=1,
FwdDfaDev::pfx_*), the rarest byte or byte pair skip (prefix=2,
FwdDfaDev::rare_*: the reference's FreqyPacked choice, literals.rs:390-510,
with a pair because one common letter is in nearly every 128-byte burst) and
the default dispatch (unset).  Kernel time of find and is_match (HIP events
on the launch stream), outputs compared.  One JSON line per pattern.
usage: python tools/prefix_ab.py [pattern ...]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import regex_amd as R  # noqa: E402
from regex_amd import _native as N  # noqa: E402
from golden_data import corpus  # noqa: E402

PATS = [r"(?i)holmes\w*", r"Sherlock\s+\w+", r"(?i)watson\w*", r"Holmes\s+\w+", r"(?i)baker\s+street",
        r"(?i)the\s+\w+", r"(?i)zqxj\w*", r">[^\n]*\n",
        # held out (round 6): not looked at when the dispatch was chosen
        r"(?i)moriarty", r"Lestrade\s+\w+", r"(?i)lady\s+\w+", r"(?i)inspector"]
MODES = [("off", "prefix=0"), ("first", "prefix=1"), ("rare", "prefix=2"), ("default", None)]


def timed(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda:0")
    text = corpus("sherlock")
    big = text * ((1 << 30) // len(text))
    n = len(big)
    hay = torch.from_numpy(np.frombuffer(big + b"\0" * 16, dtype=np.uint8).copy()).to(dev)
    for pat in sys.argv[1:] or PATS:
        res = {}
        for name, spec in MODES:
            R._debug_set(spec)
            re = R.Regex(pat)
            f = re.find_batch(hay, stride=n, length=n, count=1)
            path = N.rure_amd_last_fwd_path()
            m = re.is_match_batch(hay, stride=n, length=n, count=1)
            tf = timed(lambda: re.find_batch(hay, stride=n, length=n, count=1, out=f))
            tm = timed(lambda: re.is_match_batch(hay, stride=n, length=n, count=1, out=m))
            res[name] = (tf, tm, f.cpu().numpy(), m.cpu().numpy(), path)
        R._debug_set(None)
        same = all(np.array_equal(res["off"][k], res[x][k]) for k in (2, 3) for x in ("first", "rare", "default"))
        print(json.dumps({"pattern": pat, "bytes": n, "path": res["default"][4],
                          "find_ms": {k: round(v[0], 3) for k, v in res.items()},
                          "is_match_ms": {k: round(v[1], 3) for k, v in res.items()},
                          "find_GBps": {k: round(n / v[0] / 1e6, 1) for k, v in res.items()},
                          "outputs_equal": same}), flush=True)


if __name__ == "__main__":
    main()
