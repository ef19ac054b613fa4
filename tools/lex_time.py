"""Times the C3 strip pass (find_iter of >[^\\n]*\\n|\\n over the 2 GiB
regex-dna stream) and its lexer kernel (rure_amd_kernel_timer: HIP events
around the speculative kernel).  For A/B builds run it with
RURE_AMD_LIB_AB=librure_amd_<name>.so (Makefile target `ab`).
usage: python tools/lex_time.py [reps]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch

import regex_amd as R
from regex_amd import _native as NN
from golden_data import corpus, known_counts

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
kc = known_counts()["regexdna"]
raw = corpus("regexdna")
copies = (1 << 31) // len(raw)
L = len(raw) * copies
buf = torch.zeros(L + 16, dtype=torch.uint8, device=dev)
one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
buf[:L].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))
re = R.Regex(kc["strip"])
out = torch.empty((40_000_000, 2), dtype=torch.int64, device=dev)
cnt = torch.zeros(1, dtype=torch.int64, device=dev)
ex = torch.zeros(3, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream(dev)


def run():
    rc = NN.rure_amd_find_iter_span(re._re, ctypes.c_void_p(buf.data_ptr()), L, 0, L, None,
                                    ctypes.c_void_p(cnt.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                    out.shape[0], ctypes.c_void_p(ex.data_ptr()), ctypes.c_void_p(st.cuda_stream))
    assert rc == 0


for _ in range(5):
    run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    run()
torch.cuda.synchronize()
pass_ms = (time.perf_counter() - t0) / reps * 1e3
NN.rure_amd_kernel_timer(1)
for _ in range(reps):
    run()
n = ctypes.c_uint64(0)
ms = NN.rure_amd_kernel_timer_read(ctypes.byref(n))
NN.rure_amd_kernel_timer(0)
print({"lib": os.path.basename(NN.LIB_PATH), "matches": int(cnt.item()), "pass_ms": round(pass_ms, 4),
       "lex_kernel_ms": round(float(ms), 4), "launches": int(n.value)})
