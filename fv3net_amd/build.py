"""Build the in-tree HIP extension ``fv3net_amd/_lib/libfv3net_amd.so`` for gfx950.

Plain ``hipcc --offload-arch=gfx950 -shared`` over ``csrc/*.hip`` + ``csrc/*.cpp``;
no torch extension machinery (the C ABI has no torch types), no JIT cache: the
built ``.so`` sits in the tree so it travels to the GPU box with the snapshot.
"""
import glob
import hashlib
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "_lib")
LIB = os.path.join(LIB_DIR, "libfv3net_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("FV3_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: one rounding per operation, required for bit parity of the
# mappm / coarsen paths with the x86 reference build (no FMA there).
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", f"--offload-arch={ARCH}"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _digest():
    h = hashlib.sha256()
    for p in sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [
        os.path.join(ROOT, "include", "fv3net_amd.h")
    ]:
        with open(p, "rb") as f:
            h.update(p.encode() + f.read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile the extension if sources changed; returns the library path."""
    os.makedirs(LIB_DIR, exist_ok=True)
    stamp = LIB + ".sha256"
    digest = _digest()
    if not force and os.path.exists(LIB) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == digest:
                return LIB
    tmp = LIB + ".tmp"
    cmd = [HIPCC] + FLAGS + ["-I", os.path.join(ROOT, "include"), "-o", tmp] + sources()
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    with open(stamp, "w") as f:
        f.write(digest)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
