"""A/B of the start-state prefix skip (dfa.rs:700-711; FwdDfaDev::pfx_*,
knob prefix=0 turns it off, unset: the first-byte filter, =3: the
2-3 byte filter, pfx_depth) on sherlock text: kernel time of batched
find with and without the skip (HIP events on the launch stream), outputs
compared.  Shapes: ragged line batches (dfa_fwd_kernel, one lane per line),
fixed-stride 2000-B haystacks (tile kernel: no skip there, control) and one
long haystack (chunked long scan).  Writes one JSON line per case."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import regex_amd as R  # noqa: E402
from golden_data import corpus  # noqa: E402

PATS = [r"Sherlock\s+\w+", r"Holmes\s+\w+", r"(?i)holmes\w*", r"Baker\s+Street", r">[^\n]*\n", r"\w+@\w+",
        r"(?i)watson\w*", r"(?i)the\s+\w+", r"(?i)zqxj\w*", r"Zqxj\w*"]


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
    big = text * rep                               # ~1 GiB
    hay = torch.from_numpy(np.frombuffer(big + b"\0" * 16, dtype=np.uint8).copy()).to(dev)
    nl = np.frombuffer(big, dtype=np.uint8) == 10
    ends = np.nonzero(nl)[0] + 1
    offs = torch.from_numpy(np.concatenate([[0], ends]).astype(np.int64)).to(dev)
    nlines = offs.numel() - 1
    L = 2000
    nfix = len(big) // L
    for pat in PATS:
        out = {}
        for mode in ("0", "1", "2"):
            if mode == "1":
                R._debug_set(None)
            else:
                R._debug_set("prefix=%s" % ("3" if mode == "2" else mode))
            re = R.Regex(pat)
            r_lines = re.find_batch(hay, offsets=offs)
            t_lines = timed(lambda: re.find_batch(hay, offsets=offs, out=r_lines))
            r_fix = re.find_batch(hay, stride=L, length=L, count=nfix)
            t_fix = timed(lambda: re.find_batch(hay, stride=L, length=L, count=nfix, out=r_fix))
            r_long = re.find_batch(hay, stride=len(big), length=len(big), count=1)
            t_long = timed(lambda: re.find_batch(hay, stride=len(big), length=len(big), count=1, out=r_long), 10)
            out[mode] = (t_lines, t_fix, t_long, r_lines.cpu().numpy(), r_fix.cpu().numpy(), r_long.cpu().numpy())
        same = all(np.array_equal(out["0"][k], out[m][k]) for k in (3, 4, 5) for m in ("1", "2"))
        print(json.dumps({"pattern": pat, "match_type": R.Regex(pat).match_info()["match_type"],
                          "bytes": len(big), "lines": nlines,
                          "lines_ms": {"off": round(out["0"][0], 3), "skip": round(out["1"][0], 3)},
                          "fixed2000_ms": {"off": round(out["0"][1], 3), "skip": round(out["1"][1], 3)},
                          "long_ms": {"off": round(out["0"][2], 3), "skip1": round(out["1"][2], 3),
                                      "skip3": round(out["2"][2], 3)},
                          "outputs_equal": same}), flush=True)


if __name__ == "__main__":
    main()
