import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import numpy as np, torch
import regex_amd as R
from golden_data import corpus
from oracle_py import OracleRegex
cuda = torch.device("cuda:0")
text = corpus("sherlock")
for pat in [r"[a-z]+ing", r"\w+", r"e"]:
    n, L = 64, 9000
    buf = text[: n * L]
    re = R.Regex(pat); o = OracleRegex(re)
    d = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy()).to(cuda)
    for mode in ("burst", "nested"):
        if mode == "nested": os.environ["RURE_AMD_ITER_NESTED"] = "1"
        else: os.environ.pop("RURE_AMD_ITER_NESTED", None)
        counts, m = re.find_iter_batch(d, stride=L, length=L, count=n)
        got = [(int(a), int(b)) for a, b in m.cpu().numpy()]; k = 0
        for i in range(n):
            exp = o.find_iter(buf[i * L:(i + 1) * L]); c = int(counts[i])
            g = got[k:k + c]; k += c
            if g != exp:
                print(pat, mode, "hay", i, "missing", [x for x in exp if x not in g][:4], "extra", [x for x in g if x not in exp][:4])
    print(pat, "checked")
