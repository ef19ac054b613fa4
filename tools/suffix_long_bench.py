"""MatchType::DfaSuffix over one long haystack (a single lane
walked the whole haystack): `[a-z]+ing` and `\\w+@gmail\\.com` find /
is_match over sherlock text replicated to 1 GiB on the unit path
(launch_suffix_long) and, on a 16 MiB prefix, the one-lane path
(knob suffix_long=0), with outputs compared on the prefix.  One JSON
line per (pattern, mode)."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import regex_amd as R  # noqa: E402
from regex_amd import _native as N  # noqa: E402
from golden_data import corpus  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    text = corpus("sherlock")
    big = text * ((1 << 30) // len(text))
    n = len(big)
    hay = torch.from_numpy(np.frombuffer(big + b"\0" * 16, dtype=np.uint8).copy()).to(dev)
    small = 16 << 20
    for pat in (r"[a-z]+ing", r"\w+@gmail\.com"):
        re = R.Regex(pat)
        for mode in ("find", "is_match"):
            fn = re.find_batch if mode == "find" else re.is_match_batch
            r = fn(hay, stride=n, length=n, count=1)
            path = N.rure_amd_last_fwd_path()
            t_units = timed(lambda: fn(hay, stride=n, length=n, count=1, out=r))
            rs = fn(hay, stride=small, length=small, count=1)
            R._debug_set("suffix_long=%s" % ("0"))
            r0 = fn(hay, stride=small, length=small, count=1)
            t_lane = timed(lambda: fn(hay, stride=small, length=small, count=1, out=r0), reps=1)
            R._debug_set(None)
            print(json.dumps({"pattern": pat, "mode": mode, "bytes": n, "units_ms": round(t_units, 3),
                              "units_GBps": round(n / t_units / 1e6, 1), "path": path,
                              "one_lane_ms_16MiB": round(t_lane, 3),
                              "one_lane_GBps": round(small / t_lane / 1e6, 3),
                              "result": r.cpu().numpy().tolist(),
                              "prefix_outputs_equal": bool(np.array_equal(rs.cpu().numpy(), r0.cpu().numpy()))}),
                  flush=True)


if __name__ == "__main__":
    main()
