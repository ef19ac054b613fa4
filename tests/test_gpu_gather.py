"""rure_amd_compact_matches (the device side of the multi-GPU record gather)
against a host compaction of the same find results."""
import ctypes

import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N

pytestmark = pytest.mark.gpu


def _compact(found, base, cap):
    import torch
    rec = torch.full((max(cap, 1), 3), -7, dtype=torch.int64, device=found.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=found.device)
    rc = N.rure_amd_compact_matches(ctypes.c_void_p(found.data_ptr()), found.shape[0], base,
                                    ctypes.c_void_p(rec.data_ptr()), cap, ctypes.c_void_p(cnt.data_ptr()), None)
    assert rc == N.OK
    torch.cuda.synchronize()
    return rec.cpu().numpy(), int(cnt.item())


@pytest.mark.parametrize("n,frac", [(0, 0.0), (1, 1.0), (1000, 0.3), (1025, 0.0), (70_000, 0.01), (1 << 20, 0.5),
                                     (5_000_000, 0.001)])
def test_compact_matches(cuda, n, frac):
    import torch
    rng = np.random.default_rng(n)
    f = np.full((max(n, 1), 2), -1, dtype=np.int64)[:n]
    hit = np.sort(rng.choice(n, size=int(n * frac), replace=False)) if n else np.zeros(0, dtype=np.int64)
    f[hit, 0] = rng.integers(0, 1 << 40, size=hit.size)
    f[hit, 1] = f[hit, 0] + rng.integers(0, 100, size=hit.size)
    found = torch.from_numpy(f.copy()).to(cuda) if n else torch.empty((0, 2), dtype=torch.int64, device=cuda)
    base = 12345
    rec, cnt = _compact(found, base, max(hit.size, 1))
    assert cnt == hit.size
    exp = np.stack([hit + base, f[hit, 0], f[hit, 1]], 1) if hit.size else np.zeros((0, 3), dtype=np.int64)
    assert np.array_equal(rec[:cnt], exp)


def test_compact_capacity(cuda):
    import torch
    n = 5000
    f = np.full((n, 2), -1, dtype=np.int64)
    f[::3, 0] = 1
    f[::3, 1] = 2
    found = torch.from_numpy(f).to(cuda)
    rec, cnt = _compact(found, 0, 100)
    assert cnt == len(range(0, n, 3))
    assert np.array_equal(rec[:100, 0], np.arange(0, 300, 3))


def test_compact_find_output(cuda):
    """On the output of a batched find (the bench's C2 step)."""
    import torch
    from regex_amd.workloads import date_haystacks_host
    n, L = 4096, 256
    buf, planted = date_haystacks_host(n, L, seed=3, frac=0.1)
    re = R.Regex(r"\d{4}-\d{2}-\d{2}")
    got = re.find_batch(torch.from_numpy(buf).to(cuda), stride=L, length=L, count=n)
    rec, cnt = _compact(got, 7 * n, n)
    g = got.cpu().numpy()
    hit = np.nonzero(g[:, 0] >= 0)[0]
    assert cnt == hit.size and cnt >= len(planted)
    assert np.array_equal(rec[:cnt, 0], hit + 7 * n)
    assert np.array_equal(rec[:cnt, 1:], g[hit])
