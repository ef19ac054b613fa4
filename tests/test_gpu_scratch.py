"""Scratch memory hygiene (scratch.cpp scratch cache): device scratch kept
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
    without an explicit release.  The warm-up runs the same find_iter once:
    it loads the kernels' code objects and sizes the HIP runtime's private
    segment pool (kernels with stack frames: the fix / walk passes), which
    the runtime keeps for the process and which is not the library's."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent("""
        import gc, sys
        import numpy as np, torch
        sys.path.insert(0, %r)
        import regex_amd as R
        dev = torch.device("cuda:0")
        n, L = 64, 1 << 20
        buf = np.random.default_rng(7).choice(np.frombuffer(b"ab c\\n", dtype=np.uint8), size=n * L)

        def run():
            d = torch.from_numpy(buf).to(dev)
            re = R.Regex(r"\\w+")
            counts, m = re.find_iter_batch(d, stride=L, length=L, count=n)
            torch.cuda.synchronize()
            st = R.scratch_stats()
            k = int(counts.sum())
            del counts, m, d, re
            gc.collect(); torch.cuda.empty_cache(); torch.cuda.synchronize()
            return k, st

        k0, _ = run()
        free0, _ = torch.cuda.mem_get_info()
        assert R.scratch_stats() == {"cached": 0, "live": 0, "handles": 0}, R.scratch_stats()
        k1, st = run()
        assert k1 == k0 and st["cached"] > 0 and st["handles"] == 1, st
        free1, _ = torch.cuda.mem_get_info()
        print("free0 %%d free1 %%d" %% (free0 >> 20, free1 >> 20))
        assert R.scratch_stats() == {"cached": 0, "live": 0, "handles": 0}, R.scratch_stats()
        assert free1 >= free0 - (64 << 20), (free0 >> 20, free1 >> 20)
        print("ok")
    """ % root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
