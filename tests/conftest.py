import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    """Golden vectors extracted from the reference's ref/pytorch_reference_{single,multi}.hdf5."""
    out = {}
    for kind in ("single", "multi"):
        with np.load(os.path.join(GOLDEN, f"pytorch_reference_{kind}.npz"), allow_pickle=False) as z:
            out[kind] = {k: z[k] for k in z.files}
    with open(os.path.join(GOLDEN, "fixtures_meta.json")) as f:
        meta = json.load(f)
    for kind in out:
        out[kind]["meta"] = meta[kind]
    return out


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(GOLDEN, "kat_reference_tests.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def pkg():
    import dlrm_pkg
    return dlrm_pkg.load()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
