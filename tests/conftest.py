import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from helpers import Oracle
    return Oracle.load()


@pytest.fixture(scope="session")
def manifest():
    import json
    with open(os.path.join(TESTS, "golden", "ref", "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def H_dense(oracle, manifest):
    """Public parity matrix H regenerated from canon_tag by the oracle (pinned by H_digest)."""
    H, digest = oracle.gen_H(manifest["canon_tag"])
    assert digest.hex() == manifest["H_digest"]
    return H


@pytest.fixture(scope="session")
def engine():
    """The MI355X engine (libpvac_hip.so) — only for gpu-marked tests."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pvac_hfhe_cppbyv_amd import Engine
    return Engine(device=0)
