r"""CPU: the oracle (over the product's compiled programs) against the
Python-`re` Unicode fixtures (tests/golden/gen_unicode_fixtures.py) — the
front end's Unicode classes checked by an engine that shares none of it.
The same fixtures drive the GPU paths in test_gpu_unicode_fixtures.py."""
import gzip
import json
import os

import pytest

import regex_amd as R
from oracle_py import OracleRegex

HERE = os.path.dirname(os.path.abspath(__file__))
with gzip.open(os.path.join(HERE, "golden", "unicode_re_fixtures.json.gz"), "rt", encoding="utf-8") as _f:
    FX = json.load(_f)


def pairs(flat):
    return [(flat[i], flat[i + 1]) for i in range(0, len(flat), 2)]


def test_fixture_pool_is_multilingual():
    """The pool holds 2-, 3- and 4-byte encodings, and the generator dropped
    the code points where Python and Unicode 10 disagree (e.g. U+0301)."""
    lens = {len(c.encode()) for c in FX["pool"]}
    assert lens == {1, 2, 3, 4}
    assert "́" in FX["dropped"] and "́" not in FX["pool"]


@pytest.mark.parametrize("pat", FX["patterns"])
def test_oracle_unicode_fixtures(pat):
    o = OracleRegex(R.Regex(pat))
    for text, flat in zip(FX["ragged"] + FX["long"], FX["spans"][pat]["ragged"] + FX["spans"][pat]["long"]):
        assert o.find_iter(text.encode()) == pairs(flat), (pat, text[:40])
    for text, flat in zip(FX["stride"][:256], FX["spans"][pat]["stride"][:256]):
        assert o.find(text.encode()) == (tuple(flat) if flat else None)
