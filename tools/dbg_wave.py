import sys, zlib
sys.path.insert(0, "tests")
import numpy as np, torch
import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex
from test_gpu_iter_wave import _text, _dev
cuda = torch.device("cuda", 0)
for pat in [r"\b", r"\b\w"]:
    re = R.Regex(pat); o = OracleRegex(re)
    for chunk in (16, 61, 509, 0):
        L = 6000; count = 3
        buf = _text(zlib.crc32(pat.encode()) + 2 * 7 + 40, L * count, 40)
        for h in range(count):
            one = buf[h * L:(h + 1) * L]
            with (R.debug(iter_chunk=chunk) if chunk else R.debug(iter_wave=0)):
                c, m = re.find_iter_batch(_dev(one, cuda), stride=L, length=L, count=1)
            got = [tuple(x) for x in m.cpu().numpy().tolist()]
            exp = o.find_iter(one)
            if got != exp:
                gs, es = set(got), set(exp)
                miss = sorted(es - gs)[:6]; extra = sorted(gs - es)[:6]
                print(pat, chunk, h, len(got), len(exp), "missing", miss, "extra", extra)
                for (s, e) in miss[:3]:
                    print("   ctx", s, s // chunk, one[max(0, s - 12):s + 12])
            else:
                print(pat, chunk, h, "ok", len(got))
