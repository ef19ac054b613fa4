"""Device free memory around a large find_iter, the scratch release and a
pool trim (diagnostics for rure_amd_release_scratch)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import regex_amd as R  # noqa: E402


def free_mib(tag):
    torch.cuda.synchronize()
    f, _ = torch.cuda.mem_get_info()
    print("%-28s free %9d MiB  torch reserved %6d MiB" % (tag, f >> 20, torch.cuda.memory_reserved() >> 20),
          flush=True)
    return f


dev = torch.device("cuda:0")
torch.zeros(1, device=dev)
free_mib("start")
w = R.Regex(r"\w+")
w.find_iter_batch(torch.zeros(4096, dtype=torch.uint8, device=dev), stride=4096, length=4096, count=1)
free_mib("after warm-up")
R.release_scratch()
free_mib("after release (warm)")
n, L = 64, 1 << 20
buf = np.random.default_rng(7).choice(np.frombuffer(b"ab c\n", dtype=np.uint8), size=n * L)
d = torch.from_numpy(buf).to(dev)
free_mib("input resident")
counts, m = w.find_iter_batch(d, stride=L, length=L, count=n)
free_mib("after big find_iter")
del counts, m, d
torch.cuda.empty_cache()
free_mib("after empty_cache")
R.release_scratch()
free_mib("after release")
hip = ctypes.CDLL("libamdhip64.so")
pool = ctypes.c_void_p()
print("getpool", hip.hipDeviceGetDefaultMemPool(ctypes.byref(pool), 0))
print("trim", hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0)))
free_mib("after explicit trim")
print("devsync", hip.hipDeviceSynchronize())
print("trim2", hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0)))
free_mib("after devsync + trim")
del w
free_mib("after last free")
