"""A set of more than 64 patterns over C4's log lines: one pass for all
64-pattern groups (set_multi.hip, RURE_AMD_SET_MULTI=1) against one pass per group
(the default), and C4's 64 patterns split into G chains
(RURE_AMD_SET_CHAINS=G) against the single core-form chain; the one-pass
runs set RURE_AMD_SET_MULTI=1.
python tools/bigset_bench.py [lines] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch

import regex_amd as R
from bigset_data import SETS
from regex_amd import _native as N
from regex_amd.workloads import C4_PATTERNS, log_lines_device

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
only = sys.argv[3] if len(sys.argv) > 3 else ""
dev = torch.device("cuda:0")
buf, offs = log_lines_device(n, dev)
nbytes = int(offs[-1].item())


def run(label, pats, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        rs = R.RegexSet(pats)
        out = torch.empty((n, rs.words), dtype=torch.int64, device=dev)
        rs.matches_batch(buf, offsets=offs, out=out)
        torch.cuda.synchronize()
        path = N.rure_amd_last_fwd_path()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(reps):
            rs.matches_batch(buf, offsets=offs, out=out)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        print("%-40s %8.3f ms  %7.1f GB/s  %s" % (label, ms, nbytes / ms / 1e6, rs.multi_info()), flush=True)
        return out.cpu()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


print("lines %d, %d bytes" % (n, nbytes))
if only in ("", "big"):
    a = run("100 patterns: one pass (2 groups)", SETS[100], {"RURE_AMD_SET_MULTI": "1"})
    b = run("100 patterns: pass per group", SETS[100], {})
    print("agree", bool(torch.equal(a, b)))
if only in ("", "c4"):
    a = run("C4 64 patterns: one core chain", C4_PATTERNS, {})
    for g in (2, 3, 4):
        b = run("C4 64 patterns: %d chains" % g, C4_PATTERNS, {"RURE_AMD_SET_CHAINS": str(g), "RURE_AMD_SET_MULTI": "1"})
        print("agree", bool(torch.equal(a, b)))
