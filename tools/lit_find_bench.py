"""Literal engine vs DFA for batched find / is_match (lit_find_kernel vs the
DFA kernels): sherlock text cut into 262144 haystacks of 2000 B (~0.5 GB),
kernel times (HIP events on the launch stream) per pattern with
knob lit=0 / 1, and whether the answers agree."""
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
L, n = 2000, 262144
one = torch.from_numpy(np.frombuffer(text[: (len(text) // L) * L], dtype=np.uint8).copy()).to(dev)
buf = torch.zeros(n * L + 16, dtype=torch.uint8, device=dev)
reps = (n * L + one.numel() - 1) // one.numel()
buf[: n * L].copy_(one.repeat(reps)[: n * L])
words = sorted(set(w for w in text.decode("latin-1").split() if w.isalpha() and 5 <= len(w) <= 12))
rng = np.random.default_rng(7)
pats = {
    "Holmes": r"Holmes",
    "Sherlock|Holmes|Watson": r"Sherlock|Holmes|Watson",
    "2 rare words": "|".join(w + "zq" for w in rng.choice(words, 2, replace=False)),
    "4 words": "|".join(rng.choice(words, 4, replace=False)),
    "8 words": "|".join(rng.choice(words, 8, replace=False)),
    "16 words": "|".join(rng.choice(words, 16, replace=False)),
    "64 words": "|".join(rng.choice(words, 64, replace=False)),
    "64 rare words": "|".join(w + "zq" for w in rng.choice(words, 64, replace=False)),
}
st = torch.cuda.current_stream(dev)
for name, pat in pats.items():
    re = R.Regex(pat)
    info = re.dfa_info(0)
    res = {"pattern": name, "literals": len(re.literals() or []), "dfa_states": info and info["states"]}
    outs = {}
    for mode in ("0", "1"):
        R._debug_set("lit=%s" % (mode))
        for op in ("find", "is_match"):
            fn = re.find_batch if op == "find" else re.is_match_batch
            o = fn(buf, stride=L, length=L, count=n)
            torch.cuda.synchronize()
            path = NN.rure_amd_last_fwd_path()
            ts = []
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                fn(buf, stride=L, length=L, count=n, out=o)
                b.record(st)
                b.synchronize()
                ts.append(a.elapsed_time(b))
            outs[(mode, op)] = o.cpu()
            res["%s_%s_ms" % ("lit" if mode == "1" else "dfa", op)] = round(min(ts), 4)
            res["%s_%s_path" % ("lit" if mode == "1" else "dfa", op)] = path
    res["agree"] = bool(torch.equal(outs[("0", "find")], outs[("1", "find")]) and
                        torch.equal(outs[("0", "is_match")], outs[("1", "is_match")]))
    res["matched"] = int((outs[("1", "find")][:, 0] >= 0).sum())
    print(json.dumps(res), flush=True)
