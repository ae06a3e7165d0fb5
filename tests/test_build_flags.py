"""The product library carries no experiment knob (FV3_EXP_* / FV3_B3_EXP_*: kernel
parts replaced to price them, results invalid by construction).  CPU only: the build
flags, the guard in csrc/common.h, and the shipped .so's own build kind."""
import glob
import os
import re
import shutil
import subprocess

import pytest

from fv3net_amd import build as B

KNOB = re.compile(r"\bFV3_(?:B3_)?EXP_[A-Z0-9_]+")


def _guard_block():
    s = open(os.path.join(B.CSRC, "common.h")).read()
    a = s.index("#if defined(FV3_EXP_")
    return s[a:s.index("#endif", a)]


def test_every_knob_in_the_sources_is_guarded():
    named = set()
    for p in glob.glob(os.path.join(B.CSRC, "*")):
        if os.path.basename(p) == "common.h":
            continue
        named |= set(KNOB.findall(open(p).read()))
    guarded = set(KNOB.findall(_guard_block()))
    assert named <= guarded, f"knobs missing from common.h's product guard: {sorted(named - guarded)}"


def test_product_flags_have_no_knob():
    assert "-DFV3_PRODUCT_BUILD" in B.CFLAGS and "-DFV3_PRODUCT_BUILD" in B.FLAGS
    assert not any(KNOB.search(f) or "EXPERIMENT" in f for f in B.FLAGS)
    B.check_product_flags(env={})
    for var in B.FLAG_ENV:
        with pytest.raises(RuntimeError, match="experiment knob"):
            B.check_product_flags(env={var: "-O2 -DFV3_B3_EXP_NOMFMA"})
    with pytest.raises(RuntimeError, match="experiment knob"):
        B.check_product_flags(flags=B.CFLAGS + ["-DFV3_EXP_NOSTORE"])


def test_shipped_library_is_a_product_build():
    from fv3net_amd import _native

    if not os.path.exists(B.LIB):
        pytest.skip("library not built")
    lib = _native.load()
    assert lib.fv3_build_kind() == b"product"
    blob = open(B.LIB, "rb").read()
    assert b"experiment knobs" not in blob


@pytest.mark.skipif(shutil.which(B.HIPCC) is None and not os.path.exists(B.HIPCC), reason="no hipcc")
def test_knob_in_product_build_is_a_compile_error(tmp_path):
    src = tmp_path / "k.hip"
    src.write_text('#include "common.h"\n')
    base = [B.HIPCC, "-std=c++17", "-x", "hip", "--cuda-host-only", "-E", "-I", B.CSRC, str(src), "-o", os.devnull]
    ok = subprocess.run(base + ["-DFV3_PRODUCT_BUILD"], capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr[-2000:]
    bad = subprocess.run(base + ["-DFV3_PRODUCT_BUILD", "-DFV3_EXP_NOMFMA"], capture_output=True, text=True)
    assert bad.returncode != 0 and "product build" in bad.stderr
