"""Summarise tools/pmc_all.sh passes: per leg and kernel, mean counter values over the
last N dispatches, plus HBM bytes per launch with per-width FETCH/WRITE calibration.

    python3 tools/pmc_collect.py gpurun_out/pmc_<tag>  > summary.json

Calibration (leg `calib`, tools/calib.hip): 1 GiB read/written with 4/8/16 B per lane;
factor_w = true bytes / counted bytes.  A kernel's reads are scaled by the factor of the
width it uses (`WIDTH` below; MI355X_MICROARCH.md §HBM documents only the 16 B/lane
read factor, 2.0), writes likewise.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

N_LAST = 5
# VALU issue model (tools/valu_calib.py on the box, profiles/valu_calib.json): measured
# wave-instructions per CU per shader cycle at 8 waves/SIMD.  Full-rate class: f32
# add/mul/fma and int32 (2 cycles per wave-instruction on a SIMD-32); trans (rcp, exp,
# log, sqrt): 8 cycles; the rest the counters do not split out is compare, cndmask,
# max/min, bfe, div_scale/fmas/fixup, cvt and packed f32 (4 cycles, measured) but also
# v_mov_b32 (2 cycles, measured): the floor is given with that rest at half rate (an
# upper bound, `valu_issue_cu_cycles`) and at full rate (a lower bound, `_lo`).
VALU_RATE = {"full": 1.68, "half": 0.97, "trans": 0.49}
# read width (bytes per lane) of each kernel's dominant streams
WIDTH = {"dense_forward_kernel": 4, "dense_b3_kernel": 4, "mappm": 4, "regrid_coarsen": 4,
         "ml_epilogue_kernel": 8, "area_sums": 8, "level_sums": 4}


def short(name):
    m = re.search(r"(\w*kernel\w*|calib_\w+<[^>]*>|\w+_stage\d)", name)
    return (m.group(1) if m else name.split("(")[0])[:60]


def load_pass(d):
    """-> {kernel: [ {counter: value} per dispatch in order ]}"""
    per = defaultdict(lambda: defaultdict(dict))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row.get("Kernel_Name", ""))
                did = int(row.get("Dispatch_Id", row.get("Correlation_Id", 0)))
                c = row["Counter_Name"]
                per[k][did][c] = per[k][did].get(c, 0.0) + float(row["Counter_Value"])
    return {k: [v[i] for i in sorted(v)] for k, v in per.items()}


def width_of(k):
    for key, w in WIDTH.items():
        if key in k:
            return w
    return 16


def main(root):
    legs = {}
    for leg_dir in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(leg_dir):
            continue
        leg = os.path.basename(leg_dir)
        merged = defaultdict(dict)
        for pdir in sorted(glob.glob(os.path.join(leg_dir, "p*"))):
            if not os.path.isdir(pdir):
                continue
            for k, disp in load_pass(pdir).items():
                last = disp[-N_LAST:] if leg != "calib" else disp[-1:]
                keys = set().union(*[set(x) for x in last]) if last else set()
                for c in keys:
                    vals = [x[c] for x in last if c in x]
                    merged[k][c] = sum(vals) / len(vals)
                merged[k]["_dispatches"] = len(disp)
        legs[leg] = merged
    factors = {}
    cal = legs.get("calib", {})
    for w, tname in ((4, "float"), (8, "B8"), (16, "B16")):
        r = cal.get(f"calib_read<{tname}>", {}).get("FETCH_SIZE")
        wr = cal.get(f"calib_write<{tname}>", {}).get("WRITE_SIZE")
        factors[w] = {"read": (2 ** 30 / (r * 1024)) if r else None, "write": (2 ** 30 / (wr * 1024)) if wr else None}
    out = {"calibration": factors, "legs": {}}
    for leg, ks in legs.items():
        if leg == "calib":
            continue
        rec = {}
        for k, c in ks.items():
            w = width_of(k)
            fr = factors.get(w, {}).get("read") or 2.0
            fw = factors.get(w, {}).get("write") or 1.0
            e = dict(c)
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                e["hbm_bytes_per_launch"] = (fr * c["FETCH_SIZE"] + fw * c["WRITE_SIZE"]) * 1024
                e["read_factor"], e["write_factor"] = fr, fw
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("SQ_BUSY_CU_CYCLES"):
                e["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * c["SQ_BUSY_CU_CYCLES"])
            if "SQ_INSTS_VALU_ADD_F32" in c and "SQ_INSTS_VALU" in c:
                full = sum(c.get(n, 0.0) for n in ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
                                                    "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_INT32"))
                trans = c.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
                mfma = c.get("SQ_INSTS_MFMA", 0.0)
                half = max(0.0, c["SQ_INSTS_VALU"] - full - trans - mfma)
                e["valu_mix"] = {"full_rate": full, "half_rate": half, "trans": trans}
                # CU-cycles of VALU issue the kernel needs at the measured peaks, over the chip
                e["valu_issue_cu_cycles"] = (full / VALU_RATE["full"] + half / VALU_RATE["half"]
                                             + trans / VALU_RATE["trans"])
                e["valu_issue_cu_cycles_lo"] = (full + half) / VALU_RATE["full"] + trans / VALU_RATE["trans"]
            rec[k] = e
        out["legs"][leg] = rec
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1])
