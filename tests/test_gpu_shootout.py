"""The regex-dna shootout end to end on the device (regex_amd/shootout.py):
strip with rure_amd_replace_batch, the 9 variant counts in one fused pass,
the 11 IUB substitutions chained through rure_amd_replace_batch — the counts
and the three printed lengths must equal examples/regexdna-output.txt scaled
to the number of input copies (plus the matches across copy seams)."""
import numpy as np
import pytest

import regex_amd as R
from golden_data import corpus, known_counts
from oracle_py import OracleRegex
from regex_amd.shootout import RegexDna

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("copies", [1, 3, 64])
def test_shootout_end_to_end(cuda, copies):
    import torch
    kc = known_counts()["regexdna"]
    raw = corpus("regexdna")
    text = raw * copies
    seq = torch.from_numpy(np.frombuffer(text + b"\0" * 16, dtype=np.uint8).copy()).to(cuda)
    out = RegexDna().run(seq, len(text))
    assert out["ilen"] == kc["input_len"] * copies
    assert out["clen"] == kc["stripped_len"] * copies
    assert out["slen"] == kc["substituted_len"] * copies
    one = R.Regex(kc["strip"]).replace_all(raw, b"")
    for v, got in zip(kc["variants"], out["counts"]):
        seam = len(OracleRegex(R.Regex(v["re"])).find_iter(one * 2)) - 2 * v["count"]
        assert got == v["count"] * copies + seam * (copies - 1), v["re"]
