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


_STRUCTS = {  # header typedef -> _native ctypes mirror
    "fv3_layout": "Layout",
    "fv3_dense_desc": "DenseDesc",
    "fv3_epilogue_io": "EpilogueIO",
    "fv3_adapter_target": "AdapterTarget",
    "fv3_field": "Field",
    "fv3_nov_var": "NovVar",
    "fv3_taper_field": "TaperField",
    "fv3_strided": "Strided",
}
_RENAMED = {"inp": "in"}  # ctypes field -> C member (a Python keyword in C)


def test_ctypes_struct_layouts_match_the_header(tmp_path):
    """Every struct the host side passes by pointer has the header's size and field
    offsets (the header compiled by gcc against the ctypes mirrors)."""
    import ctypes
    import shutil
    import subprocess

    from fv3net_amd import _native

    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "fv3net_amd.h"', "int main(void) {"]
    want = {}
    for cname, pyname in _STRUCTS.items():
        cls = getattr(_native, pyname)
        want[f"{cname} sizeof"] = ctypes.sizeof(cls)
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            c_field = _RENAMED.get(fname, fname)
            want[f"{cname} {c_field}"] = getattr(cls, fname).offset
            lines.append(f'printf("{cname} {c_field} %zu\\n", offsetof({cname}, {c_field}));')
    lines += ["return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        k, v = ln.rsplit(" ", 1)
        got[k] = int(v)
    bad = {k: (got.get(k), v) for k, v in want.items() if got.get(k) != v}
    assert not bad, f"(header, ctypes) differ: {bad}"


def test_novelty_constants():
    from fv3net_amd import _native

    d = _defines(_header_text())
    assert d["FV3_NOV_MAX_VARS"] == _native.NOV_MAX_VARS
    assert d["FV3_NOV_MAX_FIELDS"] == _native.NOV_MAX_FIELDS
    assert (d["FV3_TAPER_MASK"], d["FV3_TAPER_RAMP"], d["FV3_TAPER_DECAY"]) == (
        _native.TAPER_MASK, _native.TAPER_RAMP, _native.TAPER_DECAY)
