"""The start-state prefix skip (dfa.rs:700-711, FwdDfaDev::pfx_*) cannot
change results: ragged batches (the per-lane kernel), long haystacks (the
chunked scan) and find_iter with it on equal the oracle."""
import numpy as np
import pytest

import regex_amd as R
from golden_data import corpus
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

PATS = [r"Sherlock\s+\w+", r"(?i)holmes\w*", r">[^\n]*\n", r"Baker\s+Street", r"(?:Wat|Hol)\w+",
        r"S\w+ H\w+"]


@pytest.mark.parametrize("pat", PATS)
def test_prefix_skip_lines(cuda, pat):
    import torch
    text = corpus("sherlock")[:600000]
    re = R.Regex(pat)
    o = OracleRegex(re)
    a = np.frombuffer(text, dtype=np.uint8)
    ends = np.nonzero(a == 10)[0] + 1
    offs = np.concatenate([[0], ends]).astype(np.int64)
    d = torch.from_numpy(np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    for start in (0, 1):
        got = re.find_batch(d, offsets=torch.from_numpy(offs).to(cuda), start=start).cpu().numpy()
        for i in range(len(offs) - 1):
            h = text[offs[i]:offs[i + 1]]
            e = o.find(h, start)
            g = None if got[i, 0] < 0 else (int(got[i, 0]), int(got[i, 1]))
            assert g == e, (pat, i)


@pytest.mark.parametrize("pat", PATS)
def test_prefix_skip_long(cuda, pat):
    import torch
    text = corpus("sherlock")
    re = R.Regex(pat)
    o = OracleRegex(re)
    d = torch.from_numpy(np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    for start in (0, 12345):
        got = re.find_batch(d, stride=len(text), length=len(text), count=1, start=start).cpu().numpy()
        e = o.find(text, start)
        g = None if got[0, 0] < 0 else (int(got[0, 0]), int(got[0, 1]))
        assert g == e
        assert re.is_match_batch(d, stride=len(text), length=len(text), count=1,
                                 start=start).cpu().numpy()[0] == o.is_match(text, start)
    assert re.find_iter(text[:200000]) == o.find_iter(text[:200000])
