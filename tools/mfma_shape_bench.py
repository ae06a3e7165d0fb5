"""Run tools/mfma_shape_bench.hip (tools/variants/libmfmabench.so): the split kernel's
hidden-layer loop on 16x16x32 (8 waves, 2 per SIMD) vs 32x32x16 (4 waves, 1 per SIMD)
bf16 MFMAs, one block per CU, 0-8 v_fma_f32 fillers per MFMA.  Prints the MFMA rate as a
fraction of the dense bf16 peak."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "variants", "libmfmabench.so"))
lib.mfma_shape_run.argtypes = [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
BF16_PEAK = 2516.6e12
if __name__ == "__main__":
    torch.cuda.init()
    out = torch.zeros(4096, device="cuda")
    blocks = torch.cuda.get_device_properties(0).multi_processor_count
    for rep in range(2):
        for fill in (0, 2, 4, 8):
            for shape, nch, waves, tiles, flop in ((16, 512, 8, 16, 16 * 16 * 32 * 2), (32, 1024, 4, 8, 32 * 32 * 16 * 2)):
                ms = ctypes.c_float()
                st = lib.mfma_shape_run(shape, fill, blocks, nch, 20, 96 * 1024, ctypes.c_void_p(out.data_ptr()),
                                        ctypes.byref(ms))
                assert st == 0, st
                total = blocks * nch * waves * tiles * 3 * flop
                print(f"shape {shape}x{shape} fill {fill}: {ms.value:.3f} ms  {total / (ms.value * 1e-3) / BF16_PEAK:.3f} "
                      f"of bf16 peak", flush=True)
