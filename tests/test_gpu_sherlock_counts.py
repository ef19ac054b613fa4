"""The reference's sherlock benchmark counts (bench/src/sherlock.rs, each
entry's file:line in tests/golden/known_counts.json) as GPU find_iter counts
over the corpus as one haystack — `\\w+` = 109214 (sherlock.rs:116) among
them — and `\\w+` over the corpus replicated to 1 GiB (the run engine's
workload: every copy's words plus the words merged across copy seams)."""
import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from golden_data import corpus, known_counts
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

SHERLOCK = [e for e in known_counts()["sherlock"] if e.get("corpus", "sherlock") == "sherlock"]


def _dev(t, cuda):
    import torch
    return torch.from_numpy(np.frombuffer(t + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)


@pytest.mark.parametrize("e", SHERLOCK, ids=[e["name"] for e in SHERLOCK])
def test_sherlock_count(cuda, e):
    t = corpus("sherlock")
    re = R.Regex(e["re"])
    counts, _ = re.find_iter_batch(_dev(t, cuda), stride=len(t), length=len(t), count=1)
    assert int(counts[0]) == e["count"], (e["re"], e["src"])


def test_words_one_gib(cuda):
    import torch
    t = corpus("sherlock")
    words = next(e for e in SHERLOCK if e["re"] == r"\w+")
    assert words["count"] == 109214
    copies = (1 << 30) // len(t)
    re = R.Regex(r"\w+")
    seam = len(OracleRegex(re).find_iter(t * 2)) - 2 * words["count"]
    one = torch.from_numpy(np.frombuffer(t, dtype=np.uint8).copy()).to(cuda)
    big = torch.zeros(copies * len(t) + 16, dtype=torch.uint8, device=cuda)
    big[:copies * len(t)].view(copies, len(t)).copy_(one.expand(copies, len(t)))
    n = copies * len(t)
    counts, m = re.find_iter_batch(big, stride=n, length=n, count=1, capacity=1)
    assert int(counts[0]) == copies * words["count"] + (copies - 1) * seam
    assert N.rure_amd_last_fwd_path() == -19, N.rure_amd_last_fwd_path()  # the run engine, Unicode \w
    # the first copy's records equal the oracle's
    _, m = re.find_iter_batch(big, stride=n, length=n, count=1, capacity=words["count"])
    exp = OracleRegex(re).find_iter(t)[:words["count"] - 1]
    got = [tuple(x) for x in m.cpu().numpy().tolist()][:len(exp)]
    assert got == exp
