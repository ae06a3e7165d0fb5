"""Cycles per f32 MFMA instruction on one SIMD (tools/mfma_calib.hip): 16x16x4, 4x4x1
(16 blocks) and 32x32x2, 4 independent accumulators, one wave per SIMD, in-kernel
shader-clock cycles."""
import ctypes
import os
import subprocess

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "mfma_calib.hip")
LIB = os.path.join(ROOT, "tools", "variants", "libmfma_calib.so")
if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", SRC, "-o", LIB],
                   check=True)
lib = ctypes.CDLL(LIB)
if __name__ == "__main__":
    lib.mfma_calib_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(256, device=dev)
    clk = torch.zeros(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    iters = 4000
    for op, name, flop in ((0, "v_mfma_f32_16x16x4_f32", 2048), (1, "v_mfma_f32_4x4x1_16b_f32", 512),
                           (2, "v_mfma_f32_32x32x2_f32", 4096)):
        for _ in range(2):
            lib.mfma_calib_run(op, n_cu, iters, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(clk.data_ptr()),
                               ctypes.c_void_p(s.cuda_stream))
        torch.cuda.synchronize()
        cyc = int(clk.item())
        per = cyc / (iters * 16)
        print(f"{name:28s} {per:6.2f} cycles/instruction/SIMD  {flop / per:6.1f} FLOP/cycle/SIMD", flush=True)
