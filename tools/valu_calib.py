"""Measure gfx950's VALU issue peak per instruction class (tools/valu_calib.hip).

Prints one JSON object: for each opcode and waves-per-SIMD, wave-instructions per CU per
shader cycle (the shader clock measured in-kernel), and writes it to
profiles/valu_calib.json when --out is given.  bench.py's valu_issue_frac divides a
kernel's SQ_INSTS_VALU by CUs x clock x time x the measured peak of plain VALU ops."""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "valu_calib.hip")
LIB = os.path.join(ROOT, "tools", "variants", "libvalu_calib.so")
OPS = {"v_add_f32": 0, "v_fma_f32": 1, "v_mul_f32": 2, "v_rcp_f32": 3, "v_cndmask_b32": 4, "v_pk_add_f32": 5,
       "v_pk_fma_f32": 6, "v_add_f32+v_rcp_f32": 7, "v_exp_f32": 8, "ieee_div_f32": 9,
       "v_cndmask_b32_e32": 10, "v_cmp_gt_f32": 11, "v_max_f32": 12, "v_mov_b32": 13, "v_div_scale_f32": 14,
       "v_div_fmas_f32": 15, "v_div_fixup_f32": 16, "v_add_u32": 17, "v_bfe_u32": 18}


def build():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", SRC, "-o", LIB],
                       check=True)
    return LIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--build-only", action="store_true")
    a = ap.parse_args()
    lib = ctypes.CDLL(build())
    if a.build_only:
        return
    lib.valu_calib_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(256, device=dev)
    clk = torch.zeros(2, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    res = {"n_cu": n_cu, "rates": {}}
    for name, op in OPS.items():
        per_iter = lib.valu_calib_insts_per_iter(op)
        for w in ((1, 2, 4, 8) if op < 10 else (4, 8)):
            blocks = n_cu * w
            iters = 8000 if op != 9 else 1200
            lib.valu_calib_run(op, blocks, iters, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(clk.data_ptr()),
                               ctypes.c_void_p(s.cuda_stream))
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.valu_calib_run(op, blocks, iters, ctypes.c_void_p(out.data_ptr()),
                                    ctypes.c_void_p(clk.data_ptr()), ctypes.c_void_p(s.cuda_stream))
            e1.record()
            torch.cuda.synchronize()
            if rc:
                raise RuntimeError(f"launch failed for {name}")
            ms = e0.elapsed_time(e1)
            cyc, real = (int(v) for v in clk.cpu())
            ghz = cyc / (real / 100e6) / 1e9 if real else float("nan")
            waves = blocks * 4
            insts = waves * iters * (per_iter if op != 9 else 32)
            rate = insts / (ms * 1e-3 * n_cu * ghz * 1e9)
            res["rates"].setdefault(name, {})[f"{w}_waves_per_simd"] = {
                "wave_insts_per_cu_cycle" if op != 9 else "divisions_per_cu_cycle_x64": round(rate, 4),
                "ms": round(ms, 4), "shader_ghz": round(ghz, 3)}
            print(f"{name:22s} {w} w/SIMD  {rate:7.4f} per CU-cycle  {ms:8.3f} ms  {ghz:5.3f} GHz", flush=True)
    plain = max(v["wave_insts_per_cu_cycle"] for k in ("v_add_f32", "v_fma_f32", "v_mul_f32")
                for v in res["rates"][k].values())
    res["peak_plain_valu_wave_insts_per_cu_cycle"] = plain
    print(json.dumps({"peak_plain_valu_wave_insts_per_cu_cycle": plain}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
