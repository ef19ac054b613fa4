"""Scratch memory hygiene (rure_amd.cpp scratch cache): device scratch kept
between batched calls goes back to the allocator on rure_amd_release_scratch()
and when the last rure / rure_set is freed, so the device's free memory
returns to where it was."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import regex_amd as R

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _big_find_iter(cuda):
    import torch
    n, L = 64, 1 << 20  # 64 MiB of text, dense in matches: large unit / slot scratch
    rng = np.random.default_rng(7)
    buf = rng.choice(np.frombuffer(b"ab c\n", dtype=np.uint8), size=n * L)
    d = torch.from_numpy(buf).to(cuda)
    re = R.Regex(r"\w+")
    counts, m = re.find_iter_batch(d, stride=L, length=L, count=n)
    torch.cuda.synchronize()
    return re, int(counts.sum())


def test_release_returns_device_memory(cuda):
    import torch
    torch.cuda.synchronize()
    R.release_scratch()
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    re, k = _big_find_iter(cuda)
    assert k > 0
    torch.cuda.empty_cache()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    R.release_scratch()
    torch.cuda.synchronize()
    free2, _ = torch.cuda.mem_get_info()
    # the cache held something after the call, and the release gave it back
    # (within 64 MiB: table blobs of the live regex, allocator granularity)
    assert free2 >= free1
    assert free2 >= free0 - 64 * MiB, (free0 // MiB, free1 // MiB, free2 // MiB)
    del re


def test_last_free_releases(cuda):
    """In a fresh process: freeing the last Regex returns the cached scratch
    without an explicit release."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent("""
        import gc, sys
        import numpy as np, torch
        sys.path.insert(0, %r)
        import regex_amd as R
        dev = torch.device("cuda:0")
        torch.zeros(1, device=dev); torch.cuda.synchronize()
        # warm-up (loads the kernels' code objects), then its last free
        w = R.Regex(r"\\w+")
        w.find_iter_batch(torch.zeros(4096, dtype=torch.uint8, device=dev), stride=4096, length=4096, count=1)
        torch.cuda.synchronize()
        del w
        gc.collect(); torch.cuda.empty_cache(); torch.cuda.synchronize()
        free0, _ = torch.cuda.mem_get_info()
        n, L = 64, 1 << 20
        buf = np.random.default_rng(7).choice(np.frombuffer(b"ab c\\n", dtype=np.uint8), size=n * L)
        d = torch.from_numpy(buf).to(dev)
        re = R.Regex(r"\\w+")
        counts, m = re.find_iter_batch(d, stride=L, length=L, count=n)
        torch.cuda.synchronize()
        del counts, m, d, re
        gc.collect(); torch.cuda.empty_cache(); torch.cuda.synchronize()
        free1, _ = torch.cuda.mem_get_info()
        print("free0 %%d free1 %%d" %% (free0 >> 20, free1 >> 20))
        assert free1 >= free0 - (64 << 20), (free0 >> 20, free1 >> 20)
        print("ok")
    """ % root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
