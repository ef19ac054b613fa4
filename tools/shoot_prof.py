import sys, time, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
import regex_amd as R
from regex_amd.shootout import RegexDna
from regex_amd import find_iter_span_multi
from golden_data import corpus
raw = corpus("regexdna"); copies = (1 << 31) // len(raw); N = copies * len(raw)
dev = torch.device("cuda:0")
one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
big = torch.empty(N + 16, dtype=torch.uint8, device=dev); big[:N].view(copies, len(raw)).copy_(one.expand(copies, len(raw))); big[N:] = 0
d = RegexDna()
d.run(big, N)
for rep in range(2):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    stripped, clen = d._replace(d.strip, big, N, b"", None, N); torch.cuda.synchronize(); t1 = time.perf_counter()
    res = find_iter_span_multi(d.variants, stripped, 0, clen, length=clen, capacities=[1 << 16] * 9)
    counts = [int(c.item()) for c, _, _ in res]; torch.cuda.synchronize(); t2 = time.perf_counter()
    cur, cl = stripped, clen
    ts = []
    for re_, rp in d.substs:
        a = time.perf_counter()
        cur, cl = d._replace(re_, cur, cl, rp, None, cl + cl // 4 + 1024); torch.cuda.synchronize()
        ts.append(round((time.perf_counter() - a) * 1e3, 2))
    t3 = time.perf_counter()
    print("strip %.2f ms, variants %.2f ms, substs %.2f ms %s" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, ts), flush=True)
    for re_, rp in d.substs[:2]:
        print(re_.pattern if hasattr(re_, 'pattern') else '', re_.match_info()["match_type"], flush=True)
