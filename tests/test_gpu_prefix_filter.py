"""GPU parity of the start-state prefix skip (FwdDfaDev::pfx_*; dfa.rs:700-711
prefix_at restated as a burst filter) on the chunked long scan
(last_fwd_path -4): find / is_match / shortest over long haystacks against
the oracle, with the only occurrence planted across 128-byte burst edges (a
prefix whose first byte ends a burst must not be skipped) and case-folded
prefix sets; without the skip (debug knob prefix=0), on the first byte
(prefix=1), on the rarest byte or pair of bytes (prefix=2, FwdDfaDev::rare_*)
and the default choice."""
import numpy as np
import pytest

import regex_amd as R
from regex_amd import _native as N
from oracle_py import OracleRegex

pytestmark = pytest.mark.gpu

# (pattern, an occurrence to plant)
CASES = [(r"(?i)holmes\w*", b"hOLMeszz"), (r"Sherlock\s+\w+", b"Sherlock  Holmes"), (r"(?i)baker\s+street", b"BaKeR sTreet"),
         (r"ab[cd]e\w", b"abdex"), (r"x[0-9]y", b"x7y"), (r"(?i)qu[aeiou]+z", b"QUaeZ"), (r"ab[c-h]+", b"abhh")]
L = 1 << 20


def _filler(n):
    # text rich in the prefixes' first bytes (the filter's deeper positions
    # decide), with no occurrence of any case's full prefix
    base = b"hSabxqH hoSha abaxqq QhSh Baker st bak sher xx9 " * (n // 48 + 1)
    return base[:n]


@pytest.fixture(params=[0, 1, 2, None])
def prefix_mode(request, knobs):
    if request.param is not None:
        knobs(prefix=request.param)
    yield request.param


@pytest.mark.parametrize("pat,occ", CASES)
@pytest.mark.parametrize("where", [None, 128 * 4000 - 1, 128 * 4000 - 2, 128 * 5000, 128 * 6000 + 3, L - 5])
def test_prefix_filter_long_scan(cuda, pat, occ, where, prefix_mode):
    import torch
    text = bytearray(_filler(L))
    if where is not None:
        w = min(where, L - len(occ))
        text[w:w + len(occ)] = occ
    text = bytes(text)
    re = R.Regex(pat)
    o = OracleRegex(re)
    d = torch.from_numpy(np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    f = re.find_batch(d, stride=L, length=L, count=1).cpu().numpy()
    path = N.rure_amd_last_fwd_path()
    m = re.is_match_batch(d, stride=L, length=L, count=1).cpu().numpy()
    exp = o.find(text)
    got = None if int(f[0, 0]) == -1 else (int(f[0, 0]), int(f[0, 1]))
    assert got == exp, (pat, where, got, exp)
    assert bool(m[0]) == (exp is not None)
    if re.match_info()["match_type"] == "Dfa":
        assert path == -4, pat
