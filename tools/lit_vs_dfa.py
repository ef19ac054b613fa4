"""Literal engine vs DFA for find_iter over one long haystack (sherlock
replicated to ~1 GiB): prints per-pattern kernel times (HIP events) for the
default dispatch and with knob lit=1, plus DFA sizes."""
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
from golden_data import corpus

dev = torch.device("cuda", 0)
text = corpus("sherlock")
copies = (1 << 30) // len(text)
L = copies * len(text)
buf = torch.zeros(L + 16, dtype=torch.uint8, device=dev)
one = torch.from_numpy(np.frombuffer(text, dtype=np.uint8).copy()).to(dev)
buf[:L].view(copies, len(text)).copy_(one.expand(copies, len(text)))
words = sorted(set(w for w in text.decode("latin-1").split() if w.isalpha() and 5 <= len(w) <= 12))
rng = np.random.default_rng(7)
pats = {
    "Sherlock|Holmes|Watson": r"Sherlock|Holmes|Watson",
    "16 words": "|".join(rng.choice(words, 16, replace=False)),
    "64 words": "|".join(rng.choice(words, 64, replace=False)),
    "(?i)holm": r"(?i)holm",
}
out = torch.empty((20_000_000, 2), dtype=torch.int64, device=dev)
cnt = torch.zeros(1, dtype=torch.int64, device=dev)
ex = torch.zeros(3, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream(dev)
for name, pat in pats.items():
    re = R.Regex(pat)
    info = re.dfa_info(2)
    res = {"pattern": name, "literals": len(re.literals() or []), "dfa_states": info and info["states"],
           "hot": info and info["hot"]}
    for mode in ("dfa", "lit"):
        if mode == "lit":
            R._debug_set("lit=%s" % ("1"))
        else:
            R._debug_set(None)

        def run():
            rc = NN.rure_amd_find_iter_span(re._re, ctypes.c_void_p(buf.data_ptr()), L, 0, L, None,
                                            ctypes.c_void_p(cnt.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                            out.shape[0], ctypes.c_void_p(ex.data_ptr()),
                                            ctypes.c_void_p(st.cuda_stream))
            assert rc == 0
        run()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record(st)
            run()
            b.record(st)
        torch.cuda.synchronize()
        res[mode + "_ms"] = round(float(np.median([a.elapsed_time(b) for a, b in ev])), 3)
        res[mode + "_count"] = int(cnt.item())
    print(json.dumps(res), flush=True)
