"""Lexer diagnostic: the strip pass's match count with the tail pass skipped
(RURE_AMD_LEX_TAIL=0 in the environment) vs with it, on C3's haystack.
python tools/lex_diag.py"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) == 1:
    for v in ("1", "0"):
        env = dict(os.environ, RURE_AMD_LEX_TAIL=v)
        subprocess.check_call([sys.executable, __file__, "run"], env=env)
    sys.exit(0)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
import regex_amd as R
from regex_amd import _native as NN
from golden_data import corpus, known_counts
kc = known_counts()["regexdna"]
raw = corpus("regexdna")
copies = 2000
L = len(raw) * copies
dev = torch.device("cuda", 0)
buf = torch.zeros(L + 16, dtype=torch.uint8, device=dev)
one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
buf[:L].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))
re = R.Regex(kc["strip"])
counts, m = re.find_iter_batch(buf, stride=L, length=L, count=1)
mm = m.cpu().numpy()
print("LEX_TAIL=%s matches %d first %s" % (os.environ.get("RURE_AMD_LEX_TAIL"), int(counts[0]), mm[:3].tolist()))
