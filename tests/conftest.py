import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def set_variant(monkeypatch, name: str, value: str) -> None:
    """Select a kernel variant for one test: the library reads variant selectors only
    while FV3_VARIANTS=1 (csrc/common.h variant_env, _native.variant)."""
    monkeypatch.setenv("FV3_VARIANTS", "1")
    monkeypatch.setenv(name, value)


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fv3net_amd import _native

    _native.load()
    return torch.device("cuda", 0)
