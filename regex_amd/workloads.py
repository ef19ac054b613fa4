"""Synthetic, seeded haystack batches for the BASELINE.json configurations
(SURVEY.md §8d).  Generated on the device so the 4 GiB / 16 GiB batches never
cross PCIe; small batches for parity tests can be generated on the host with
the same recipe (numpy) and copied over.

C1/C2 recipe: printable ASCII (0x20-0x7E) with ~20 % digits (to exercise
partial date matches); a fraction of the haystacks gets one planted
`YYYY-MM-DD` at a uniform offset.
"""
import numpy as np

DATE_LEN = 10


def _plant_dates_np(buf, n, L, frac, rng):
    k = int(round(n * frac))
    idx = rng.choice(n, size=k, replace=False) if k else np.zeros(0, dtype=np.int64)
    offs = rng.integers(0, max(L - DATE_LEN, 0) + 1, size=k)
    digits = rng.integers(0, 10, size=(k, DATE_LEN)).astype(np.uint8) + ord("0")
    digits[:, 4] = ord("-")
    digits[:, 7] = ord("-")
    for j in range(k):
        o = int(idx[j]) * L + int(offs[j])
        buf[o:o + DATE_LEN] = digits[j]
    return np.sort(idx)


def date_haystacks_host(n, L, seed, frac=0.01, digit_frac=0.2):
    """Host (numpy) batch: n x L bytes, fixed stride L."""
    rng = np.random.default_rng(seed)
    r = rng.integers(0, 1 << 31, size=n * L, dtype=np.int64)
    is_digit = (r % 1000) < int(digit_frac * 1000)
    v = (r >> 10)
    buf = np.where(is_digit, ord("0") + v % 10, 0x20 + v % 95).astype(np.uint8)
    planted = _plant_dates_np(buf, n, L, frac, rng)
    return buf, planted


def date_haystacks_device(n, L, seed, device, frac=0.01, digit_frac=0.2, chunk=1 << 28):
    """Device (torch) batch of the same recipe; returns (uint8 tensor, planted idx)."""
    import torch
    total = n * L
    out = torch.empty(total, dtype=torch.uint8, device=device)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    for s in range(0, total, chunk):
        e = min(total, s + chunk)
        r = torch.randint(0, 1 << 31, (e - s,), generator=g, device=device, dtype=torch.int64)
        is_digit = (r % 1000) < int(digit_frac * 1000)
        v = r >> 10
        out[s:e] = torch.where(is_digit, 48 + v % 10, 32 + v % 95).to(torch.uint8)
        del r, is_digit, v
    rng = np.random.default_rng(seed ^ 0x5EED)
    k = int(round(n * frac))
    idx = np.sort(rng.choice(n, size=k, replace=False)) if k else np.zeros(0, dtype=np.int64)
    offs = rng.integers(0, max(L - DATE_LEN, 0) + 1, size=k)
    digits = rng.integers(0, 10, size=(k, DATE_LEN)).astype(np.uint8) + ord("0")
    digits[:, 4] = ord("-")
    digits[:, 7] = ord("-")
    if k:
        pos = torch.from_numpy((idx * L + offs)[:, None] + np.arange(DATE_LEN)[None, :]).to(device)
        out[pos.reshape(-1)] = torch.from_numpy(digits.reshape(-1)).to(device)
    return out, idx
