"""Device free memory at each step of test_gpu_scratch.test_last_free_releases
with the library's scratch bookkeeping (rure_amd_scratch_stats)."""
import gc
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import regex_amd as R  # noqa: E402

dev = torch.device("cuda:0")


def show(tag):
    gc.collect()
    torch.cuda.empty_cache()
    torch.cuda.synchronize()
    f, _ = torch.cuda.mem_get_info()
    print("%-24s free %8d MiB  torch alloc %5d MiB reserved %5d MiB  %s" %
          (tag, f >> 20, torch.cuda.memory_allocated() >> 20, torch.cuda.memory_reserved() >> 20,
           R.scratch_stats()), flush=True)


torch.zeros(1, device=dev)
show("start")
w = R.Regex(r"\w+")
w.find_iter_batch(torch.zeros(4096, dtype=torch.uint8, device=dev), stride=4096, length=4096, count=1)
show("warm-up")
del w
show("warm-up freed")
n, L = 64, 1 << 20
buf = np.random.default_rng(7).choice(np.frombuffer(b"ab c\n", dtype=np.uint8), size=n * L)
d = torch.from_numpy(buf).to(dev)
show("input")
re = R.Regex(r"\w+")
show("compiled")
counts, m = re.find_iter_batch(d, stride=L, length=L, count=n)
show("find_iter")
print("matches", m.shape, flush=True)
del counts, m
show("outputs freed")
del d
show("input freed")
del re
show("regex freed")
re2 = R.Regex(r"\w+")
d = torch.from_numpy(buf).to(dev)
counts, m = re2.find_iter_batch(d, stride=L, length=L, count=n)
del counts, m, d
show("second run")
R.release_scratch()
show("released")
del re2
show("last free")
