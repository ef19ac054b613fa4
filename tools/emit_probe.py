"""Strip-pass find_iter_span over the C3 raw text with and without its
header lines ('>' replaced), for kernel traces of the post passes:
python tools/emit_probe.py [hdr|nohdr] [REPS]"""
import ctypes
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

mode = sys.argv[1] if len(sys.argv) > 1 else "hdr"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
kc = known_counts()["regexdna"]
unit = corpus("regexdna")
if mode == "nohdr":
    unit = unit.replace(b">", b"a")
copies = (1 << 31) // len(unit)
L = len(unit) * copies
buf = torch.zeros(L + 16, dtype=torch.uint8, device=dev)
one = torch.from_numpy(np.frombuffer(unit, dtype=np.uint8).copy()).to(dev)
buf[:L].view(copies, len(unit)).copy_(one.expand(copies, len(unit)))
re = R.Regex(kc["strip"])
out = torch.empty((40_000_000, 2), dtype=torch.int64, device=dev)
cnt = torch.zeros(1, dtype=torch.int64, device=dev)
ex = torch.zeros(3, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream(dev)
for _ in range(reps):
    rc = NN.rure_amd_find_iter_span(re._re, ctypes.c_void_p(buf.data_ptr()), L, 0, L, None,
                                    ctypes.c_void_p(cnt.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                    out.shape[0], ctypes.c_void_p(ex.data_ptr()), ctypes.c_void_p(st.cuda_stream))
    assert rc == 0
torch.cuda.synchronize()
print(mode, int(cnt.item()))
