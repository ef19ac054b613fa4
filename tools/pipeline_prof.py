"""The C3 shootout pipeline (regex_amd/shootout.py) stage by stage: the
strip replace_all, the fused variant pass and each IUB replace_all timed on
the host with a device sync after each (warm, median of --reps runs), plus
the number of matches each substitution replaced.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.
usage: python tools/pipeline_prof.py [--reps N]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from regex_amd import shootout  # noqa: E402
from regex_amd import find_iter_span_multi  # noqa: E402
import regex_amd as R  # noqa: E402
from golden_data import corpus  # noqa: E402

reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 5
dev = torch.device("cuda:0")
raw = corpus("regexdna")
copies = (1 << 31) // len(raw)
N = copies * len(raw)
one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
big = torch.empty(N + 16, dtype=torch.uint8, device=dev)
big[:N].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))
big[N:] = 0
dna = shootout.RegexDna()


def stage(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, (time.perf_counter() - t) * 1e3


rows = []
for rep in range(reps + 1):
    row = {}
    (stripped, clen), row["strip"] = stage(lambda: dna._replace(dna.strip, big, N, b"", None, N))
    _, row["variants"] = stage(lambda: find_iter_span_multi(dna.variants, stripped, 0, clen, length=clen,
                                                            capacities=[1 << 16] * 9))
    cap = 2 * clen + 4096  # (as regex_amd/shootout.py: the stream grows by a third)
    (_, lengths), row["iub_chain"] = stage(lambda: R.replace_all_chain([r for r, _ in dna.substs],
                                                                       [t for _, t in dna.substs], stripped,
                                                                       length=clen, capacity=cap))
    lens = lengths.cpu().numpy().tolist()
    cl = lens[-1]
    assert cl <= cap
    row["_grow"] = [b - a for a, b in zip(lens[:-1], lens[1:])]
    if rep:
        rows.append(row)
keys = [k for k in rows[0] if not k.startswith("_")]
med = {k: round(float(np.median([r[k] for r in rows])), 3) for k in keys}
print(json.dumps({"stage_ms": med, "total_ms": round(sum(med.values()), 3), "lengths": [N, clen, cl],
                  "iub_growth_bytes": rows[0]["_grow"]}), flush=True)
