"""Tuning sweep for the chunked find_iter (C3 passes): times the strip pass
and the 9 variant passes (HIP events on the launch stream) under each
iter_bs / iter_lanes debug-knob setting given on the command line,
e.g.  python tools/iter_sweep.py 256:1024 1024:2048 256:1024:NESTED"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch

import regex_amd as R
from regex_amd import _native as NN
from golden_data import corpus, known_counts

dev = torch.device("cuda", 0)
kc = known_counts()["regexdna"]
raw = corpus("regexdna")
copies = (1 << 31) // len(raw)
N = copies * len(raw)
one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
big = torch.zeros(N + 16, dtype=torch.uint8, device=dev)
big[:N].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))
seq1 = R.Regex(kc["strip"]).replace_all(raw, b"")
M = len(seq1) * copies
seq = torch.zeros(M + 16, dtype=torch.uint8, device=dev)
s1 = torch.from_numpy(np.frombuffer(seq1, dtype=np.uint8).copy()).to(dev)
seq[:M].view(copies, len(seq1)).copy_(s1.expand(copies, len(seq1)))
out = torch.empty((40_000_000, 2), dtype=torch.int64, device=dev)
cnt = torch.zeros(1, dtype=torch.int64, device=dev)
ex = torch.zeros(3, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream(dev)
passes = [("strip", R.Regex(kc["strip"]), big, N)] + [(v["re"], R.Regex(v["re"]), seq, M) for v in kc["variants"]]


def run(re_, buf, L):
    rc = NN.rure_amd_find_iter_span(re_._re, ctypes.c_void_p(buf.data_ptr()), L, 0, L, None,
                                    ctypes.c_void_p(cnt.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                    out.shape[0], ctypes.c_void_p(ex.data_ptr()), ctypes.c_void_p(st.cuda_stream))
    assert rc == 0


for cfg in sys.argv[1:] or ["1024:2048"]:
    parts = cfg.split(":")
    bs, lanes = parts[0], parts[1]
    R._debug_set("iter_bs=%s,iter_lanes=%s" % (bs, lanes))
    res = {}
    for name, re_, buf, L in passes:
        for _ in range(2):
            run(re_, buf, L)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record(st)
            run(re_, buf, L)
            b.record(st)
        torch.cuda.synchronize()
        res[name] = (round(float(np.median([a.elapsed_time(b) for a, b in ev])), 3), int(cnt.item()))
    tot = sum(v[0] for v in res.values())
    print(json.dumps({"cfg": cfg, "total_ms": round(tot, 3), "passes": res}), flush=True)
