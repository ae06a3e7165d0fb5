"""The drop-in boundary on CPU (no GPU calls): the HIP extension builds, loads, and
exports every entry point include/fv3net_amd.h declares, with the ABI version and the
enum values the Python host side uses."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fv3net_amd.h")


def _header_text():
    with open(HEADER) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)  # block comments
    return re.sub(r"//[^\n]*", "", text)


def _declared_functions(text):
    # a declaration starts a line with its return type and names an fv3_ function
    return sorted(set(re.findall(r"^[a-z][\w \*]*?\b(fv3_\w+)\s*\(", text, flags=re.M)))


def _defines(text):
    return {k: int(v, 0) for k, v in re.findall(r"^#define\s+(FV3_\w+)\s+(-?(?:0x)?[0-9a-fA-F]+)\b", text, flags=re.M)}


@pytest.fixture(scope="module")
def lib():
    import ctypes

    from fv3net_amd import build

    return ctypes.CDLL(build.build())


def test_header_declares_the_entry_points():
    names = _declared_functions(_header_text())
    assert len(names) > 30
    for must in ("fv3_dense_create", "fv3_dense_forward", "fv3_dense_forward_ex", "fv3_dense_destroy",
                 "fv3_mappm", "fv3_last_error", "fv3_abi_version"):
        assert must in names, must


def test_library_exports_every_declared_function(lib):
    missing = [n for n in _declared_functions(_header_text()) if not hasattr(lib, n)]
    assert not missing, f"declared in include/fv3net_amd.h but not exported: {missing}"


def test_python_signatures_cover_exported_symbols(lib):
    from fv3net_amd import _native

    declared = set(_declared_functions(_header_text()))
    for name in _native.EXPORTED_SYMBOLS:
        assert name in declared, f"{name} is bound in _native.py but not declared in the header"
        assert hasattr(lib, name), name


def test_abi_version_and_constants_match_the_header(lib):
    from fv3net_amd import _native

    d = _defines(_header_text())
    assert lib.fv3_abi_version() == _native.ABI_VERSION
    assert d["FV3_DENSE_F32"] == _native.DENSE_F32
    assert d["FV3_DENSE_BF16X3"] == _native.DENSE_BF16X3
    assert d["FV3_DENSE_BF16X6"] == _native.DENSE_BF16X6
    assert d["FV3_OK"] == _native.FV3_OK
