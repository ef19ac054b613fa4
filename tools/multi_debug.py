"""Diagnostics of the one-pass multi-group set kernel: RURE_AMD_MULTI_DEBUG
output for C4's patterns split into 2..4 chains."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["RURE_AMD_MULTI_DEBUG"] = "1"
os.environ["RURE_AMD_SET_MULTI"] = "1"
import numpy as np
import torch

import regex_amd as R
from regex_amd.workloads import C4_PATTERNS, log_lines_host

buf, offs = log_lines_host(3000, seed=1)
d = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).cuda()
for g in (2, 3, 4):
    os.environ["RURE_AMD_SET_CHAINS"] = str(g)
    rs = R.RegexSet(C4_PATTERNS)
    rs.matches_batch(d, offsets=torch.from_numpy(offs).cuda())
    torch.cuda.synchronize()
    print(g, rs.multi_info(), flush=True)
