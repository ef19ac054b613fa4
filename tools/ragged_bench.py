"""Ragged single-regex batches: the sherlock text
replicated to ~1 GiB and cut at its newlines (23.5 M lines), batched find /
is_match per line through the offsets API.  Kernel time by HIP events on the
launch stream for the line kernel (dfa_line_kernel, default) and the previous
one-lane-per-haystack kernel (knob lines=0); outputs compared.  One JSON
line per (pattern, mode)."""
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

PATS = [r"Sherlock\s+\w+", r"\d{4}-\d{2}-\d{2}", r"\w+@\w+\.\w+", r"(?i)watson", r"Holmes\s+\w+"]


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


def main():
    dev = torch.device("cuda:0")
    text = corpus("sherlock")
    rep = (1 << 30) // len(text)
    big = text * rep
    hay = torch.from_numpy(np.frombuffer(big + b"\0" * 16, dtype=np.uint8).copy()).to(dev)
    ends = np.nonzero(np.frombuffer(big, dtype=np.uint8) == 10)[0] + 1
    offs = torch.from_numpy(np.concatenate([[0], ends]).astype(np.int64)).to(dev)
    nlines = offs.numel() - 1
    nbytes = int(ends[-1])
    for pat in PATS:
        re = R.Regex(pat)
        res = {}
        for lines in ("1", "0"):
            R._debug_set("lines=%s" % (lines))
            for mode in ("find", "is_match"):
                fn = re.find_batch if mode == "find" else re.is_match_batch
                r = fn(hay, offsets=offs)
                path = N.rure_amd_last_fwd_path()
                t = timed(lambda: fn(hay, offsets=offs, out=r))
                res[(lines, mode)] = (t, r.cpu().numpy(), path)
        R._debug_set(None)
        for mode in ("find", "is_match"):
            t1, r1, p1 = res[("1", mode)]
            t0, r0, p0 = res[("0", mode)]
            print(json.dumps({"pattern": pat, "mode": mode, "match_type": re.match_info()["match_type"],
                              "lines": nlines, "bytes": nbytes,
                              "line_kernel_ms": round(t1, 4), "line_kernel_GBps": round(nbytes / t1 / 1e6, 1),
                              "path": p1, "per_lane_ms": round(t0, 4),
                              "per_lane_GBps": round(nbytes / t0 / 1e6, 1), "path_off": p0,
                              "outputs_equal": bool(np.array_equal(r1, r0)),
                              "matches": int((r1[:, 1] >= 0).sum()) if r1.ndim == 2 else int(r1.sum())}),
                  flush=True)


if __name__ == "__main__":
    main()
