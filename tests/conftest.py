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


def require_variant_kernels() -> None:
    """Skip unless the loaded library holds the variant kernels (csrc/common.h
    FV3_VARIANT_KERNELS: tools/ variant builds only; the product library keeps the kernels
    its own heuristics pick)."""
    from fv3net_amd import _native

    if _native.load().fv3_build_kind() == b"product":
        pytest.skip("variant kernel: not in the product library (tools/build_variant.sh builds it)")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fv3net_amd import _native

    _native.load()
    return torch.device("cuda", 0)
