import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP kernels)")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture
def knobs():
    """Debug-only engine overrides for one test (regex_amd.debug's table;
    names in regex_amd/csrc/host/knobs.hpp): knobs(lit=1) replaces the
    table, knobs() clears it; cleared again after the test."""
    import regex_amd as R

    def set_(**kw):
        R._debug_set(",".join("%s=%d" % (k, int(v)) for k, v in kw.items()) or None)

    yield set_
    R._debug_set(None)
