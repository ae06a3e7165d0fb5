"""Build the in-tree HIP extension ``fv3net_amd/_lib/libfv3net_amd.so`` for gfx950.

Plain ``hipcc --offload-arch=gfx950``: each ``csrc/*.hip`` / ``csrc/*.cpp`` compiles to
its own object (in parallel, cached by content hash under ``_lib/obj``), then one
``-shared`` link.  No torch extension machinery (the C ABI has no torch types), no JIT
cache: the built ``.so`` sits in the tree so it travels to the GPU box with the snapshot.
"""
import concurrent.futures
import glob
import hashlib
import os
import re
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "_lib")
OBJ_DIR = os.path.join(LIB_DIR, "obj")
LIB = os.path.join(LIB_DIR, "libfv3net_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("FV3_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: one rounding per operation, required for bit parity of the
# mappm / coarsen paths with the x86 reference build (no FMA there).
# FV3_PRODUCT_BUILD: csrc/common.h refuses every experiment knob (FV3_EXP_*, results
# invalid by construction) in this build; those compile only in tools/ variant builds.
CFLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", f"--offload-arch={ARCH}", "-DFV3_PRODUCT_BUILD"]
FLAGS = CFLAGS + ["-shared"]
# environment variables hipcc / clang read extra flags from
FLAG_ENV = ("HIPCC_COMPILE_FLAGS_APPEND", "HIPCC_LINK_FLAGS_APPEND", "HIPFLAGS", "CXXFLAGS", "CPPFLAGS")
_EXP = re.compile(r"FV3_\w*EXP|FV3_EXPERIMENT")


def check_product_flags(flags=None, env=None) -> None:
    """Refuse an experiment knob anywhere in the product build's flags."""
    env = os.environ if env is None else env
    texts = [" ".join(CFLAGS if flags is None else flags)] + [env.get(k, "") for k in FLAG_ENV]
    for t in texts:
        m = _EXP.search(t)
        if m:
            raise RuntimeError(f"experiment knob {m.group(0)!r} in the product build flags: build variants with "
                               "tools/build_*variant.sh")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "include", "fv3net_amd.h")]


def _read(p):
    with open(p, "rb") as f:
        return f.read()


_INC_HIP = re.compile(rb'#include\s+"([^"/]+\.hip)"')


def _obj_digest(src, hdr_blob):
    h = hashlib.sha256()
    h.update(_read(src) + hdr_blob + " ".join(CFLAGS).encode())
    # a *_fast.hip unit includes its exact sibling's source (csrc/mappm_fast.hip)
    for inc in _INC_HIP.findall(_read(src)):
        h.update(_read(os.path.join(CSRC, inc.decode())))
    return h.hexdigest()[:20]


def _digest():
    h = hashlib.sha256()
    for p in sources() + _headers():
        h.update(p.encode() + _read(p))
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()


def _compile(src, obj, verbose):
    cmd = [HIPCC] + CFLAGS + ["-I", os.path.join(ROOT, "include"), "-c", src, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile the extension if sources changed; returns the library path."""
    check_product_flags()
    os.makedirs(OBJ_DIR, exist_ok=True)
    stamp = LIB + ".sha256"
    digest = _digest()
    if not force and os.path.exists(LIB) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == digest:
                return LIB
    hdr_blob = b"".join(_read(p) for p in _headers())
    objs, todo = [], []
    for src in sources():
        base = os.path.splitext(os.path.basename(src))[0]
        obj = os.path.join(OBJ_DIR, f"{base}.{_obj_digest(src, hdr_blob)}.o")
        objs.append(obj)
        if force or not os.path.exists(obj):
            todo.append((src, obj))
    jobs = max(1, min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 8))
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        for f in [ex.submit(_compile, s, o, verbose) for s, o in todo]:
            f.result()
    keep = set(objs)
    for stale in glob.glob(os.path.join(OBJ_DIR, "*.o")):
        if stale not in keep:
            os.remove(stale)
    tmp = LIB + ".tmp"
    cmd = [HIPCC] + FLAGS + ["-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    with open(stamp, "w") as f:
        f.write(digest)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
