"""Driver for per-kernel PMC passes (tools/pmc_all.sh): run ONE bench leg N times.

    python3 tools/pmc_drive.py <leg> <n>

Legs are the kernels bench.py reports (its headline + every `extra` entry):
  dense_c48, dense_c384, dense_c384_bf16x3, emulator_c384 (bf16x3), emulator_c384_f32,
  mappm_c384_k1, mappm_c384_k10, mappm_c12, coarsen_1f, coarsen_4f, stepper_c96,
  predict_mappm_c384, and the bf16x6 legs dense_c48_bf16x6, dense_c384_bf16x6,
  emulator_c384_bf16x6, predict_mappm_c384_bf16x6.
Each leg warms up (untimed) before its N profiled launches; the collector keeps only the
last N dispatches of the leg's dominant kernel.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402


def make(leg, dev):
    if leg == "dense_c48":
        return W.make_dense_workload(48, seed=1, device=dev)
    if leg == "dense_c384":
        return W.make_dense_workload(384, seed=3, device=dev)
    if leg == "dense_c384_bf16x3":
        return W.make_dense_workload(384, seed=3, device=dev, precision="bf16x3")
    if leg in ("dense_c48_bf16x6", "dense_c384_bf16x6"):
        return W.make_dense_workload(48 if "c48" in leg else 384, seed=3, device=dev, precision="bf16x6")
    if leg == "emulator_c384_bf16x6":
        return W.make_emulator_workload(384, seed=13, device=dev, precision="bf16x6")
    if leg == "predict_mappm_c384_bf16x6":
        return W.make_predict_mappm_workload(384, seed=17, device=dev, precision="bf16x6")
    if leg == "emulator_c384":
        return W.make_emulator_workload(384, seed=13, device=dev, precision="bf16x3")
    if leg == "emulator_c384_f32":
        return W.make_emulator_workload(384, seed=13, device=dev, precision="f32")
    if leg == "mappm_c384_k1":
        return W.make_mappm_workload(W.c_columns(384), 79, 79, 1, seed=5, device=dev)
    if leg == "mappm_c384_k10":
        return W.make_mappm_workload(W.c_columns(384), 79, 79, 10, seed=5, device=dev)
    if leg in ("mappm_c384_k1_exact", "mappm_c384_k10_exact"):
        return W.make_mappm_workload(W.c_columns(384), 79, 79, 1 if "k1_" in leg else 10, seed=5, device=dev,
                                     exact=True)
    if leg in ("coarsen_1f_exact", "coarsen_4f_exact"):
        return W.make_coarsen_workload(384, 8, 1 if "1f" in leg else 4, seed=7, device=dev, exact=True)
    if leg == "mappm_c12":
        return W.make_mappm_workload(W.c_columns(12), 79, 50, 1, seed=5, device=dev)
    if leg == "coarsen_0f":  # pass 1 only (coarse delp / phalf, denominators)
        return W.make_coarsen_workload(384, 8, 0, seed=7, device=dev)
    if leg == "coarsen_1f":
        return W.make_coarsen_workload(384, 8, 1, seed=7, device=dev)
    if leg == "coarsen_4f":
        return W.make_coarsen_workload(384, 8, 4, seed=7, device=dev)
    if leg == "stepper_c96":
        return W.make_stepper_workload(96, seed=11, device=dev)
    if leg == "predict_mappm_c384" and hasattr(W, "make_predict_mappm_workload"):
        return W.make_predict_mappm_workload(384, seed=17, device=dev)
    # one rank's share of the 8-GPU decompositions (bench.py rank_share_legs)
    if leg == "stepper_c96_r8":
        return W.make_sharded_stepper_workload(96, 0, 8, seed=11, device=dev, stub_exchange=True)
    if leg in ("emulator_c384_r8", "emulator_c384_f32_r8"):
        return W.make_emulator_workload(384, seed=13, device=dev, precision="f32" if "f32" in leg else "bf16x3",
                                        world=8)
    if leg in ("predict_mappm_c384_r8", "predict_mappm_c384_bf16x6_r8"):
        return W.make_predict_mappm_workload(384, 0, 8, seed=21, device=dev,
                                             precision="bf16x6" if "bf16x6" in leg else "f32")
    raise SystemExit(f"unknown leg {leg}")


def calib(dev, n):
    """Known byte counts per access width (tools/calib.hip): 1 GiB, past the 256 MiB
    Infinity Cache, read and written at 4, 8 and 16 B per lane."""
    import ctypes

    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants", "libcalib.so"))
    lib.calib_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                              ctypes.c_void_p]
    nbytes = 1 << 30
    buf = torch.zeros(nbytes // 4, device=dev)
    out = torch.zeros(4, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(n):
        for width in (4, 8, 16):
            for write in (0, 1):
                assert lib.calib_run(width, write, buf.data_ptr(), nbytes, out.data_ptr(), st) == 0
    torch.cuda.synchronize()
    print(f"calib: {n} rounds of {nbytes} B per kernel", flush=True)


if __name__ == "__main__":
    leg, n = sys.argv[1], int(sys.argv[2])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if leg == "calib":
        calib(dev, n)
        sys.exit(0)
    wl = make(leg, dev)
    for _ in range(3):
        wl.step()
    torch.cuda.synchronize()
    for _ in range(n):
        wl.step()
    torch.cuda.synchronize()
    print(f"{leg}: {n} steps done", flush=True)
