"""Publish a tools/pmc_all.sh run into profiles/:

    python3 tools/pmc_publish.py gpurun_out/pmc_<tag> <tag>

* profiles/<tag>_pmc/<leg>/p<N>.csv   the counter rows of the product kernels (and the
                                       calibration kernels), straight from rocprofv3
* profiles/<tag>_pmc_summary.json     tools/pmc_collect.py's per-leg, per-kernel means
* profiles/pmc_traffic.json           per bench leg: the dominant kernel's HBM bytes per
                                       launch and its MFMA / VALU counters (bench.py
                                       attaches `traffic` from here to every leg)
"""
import csv
import glob
import io
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

# bench leg -> (pmc_drive leg, dominant kernel short name)
LEGS = {
    "dense_c48": ("dense_c48", "dense_forward_kernel"),
    "dense_c384": ("dense_c384", "dense_forward_kernel"),
    "dense_c384_bf16x3": ("dense_c384_bf16x3", "dense_b3_kernel"),
    "emulator_c384": ("emulator_c384", "dense_b3_kernel"),
    "emulator_c384_f32": ("emulator_c384_f32", "dense_forward_kernel"),
    "mappm_c384_79to79_kord1": ("mappm_c384_k1", "mappm_ppm_kernel"),
    "mappm_c384_79to79_kord10": ("mappm_c384_k10", "mappm_cs_global_kernel"),
    "mappm_c12_79to50_kord1": ("mappm_c12", "mappm_ppm_levels_kernel"),
    "mappm_c384_79to79_kord1_exact": ("mappm_c384_k1_exact", "mappm_ppm_kernel"),
    "mappm_c384_79to79_kord10_exact": ("mappm_c384_k10_exact", "mappm_cs_global_kernel"),
    "coarsen_c384_to_c48_1field_exact": ("coarsen_1f_exact", "regrid_coarsen_cells_kernel"),
    "coarsen_c384_to_c48_4field_exact": ("coarsen_4f_exact", "regrid_coarsen_cells_kernel"),
    "coarsen_c384_to_c48_1field": ("coarsen_1f", "regrid_coarsen_cells_kernel"),
    "coarsen_c384_to_c48_4field": ("coarsen_4f", "regrid_coarsen_cells_kernel"),
    "stepper_c96": ("stepper_c96", "ml_epilogue_kernel"),
    "stepper_c96_predict": ("stepper_c96", "dense_forward_kernel"),
    "predict_mappm_c384": ("predict_mappm_c384", "dense_forward_kernel"),
    "predict_mappm_c384_mappm": ("predict_mappm_c384", "mappm_ppm_pair_kernel"),
    "dense_c48_bf16x6": ("dense_c48_bf16x6", "dense_b3_kernel"),
    "dense_c384_bf16x6": ("dense_c384_bf16x6", "dense_b3_kernel"),
    "emulator_c384_bf16x6": ("emulator_c384_bf16x6", "dense_b3_kernel"),
    "predict_mappm_c384_bf16x6": ("predict_mappm_c384_bf16x6", "dense_b3_kernel"),
    "stepper_c96_rank_of_8": ("stepper_c96_r8", "dense_forward_kernel"),
    "emulator_c384_rank_of_8": ("emulator_c384_r8", "dense_b3_kernel"),
    "emulator_c384_rank_of_8_f32": ("emulator_c384_f32_r8", "dense_forward_kernel"),
    "predict_mappm_c384_rank_of_8": ("predict_mappm_c384_r8", "dense_forward_kernel"),
    "predict_mappm_c384_rank_of_8_bf16x6": ("predict_mappm_c384_bf16x6_r8", "dense_b3_kernel"),
    "predict_mappm_c384_rank_of_8_mappm": ("predict_mappm_c384_r8", "mappm_ppm_pair_split_kernel"),
}
KEEP = ("fv3::", "calib_")


def main(src, tag):
    out_dir = os.path.join(ROOT, "profiles", f"{tag}_pmc")
    for path in glob.glob(os.path.join(src, "*", "p*", "*counter_collection.csv")):
        leg = os.path.basename(os.path.dirname(os.path.dirname(path)))
        pas = os.path.basename(os.path.dirname(path))
        with open(path) as f:
            rows = list(csv.DictReader(f))
        if not rows:
            continue
        keep = [r for r in rows if any(k in r.get("Kernel_Name", "") for k in KEEP)]
        os.makedirs(os.path.join(out_dir, leg), exist_ok=True)
        with open(os.path.join(out_dir, leg, f"{pas}.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(keep)
    summary = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_collect.py"), src],
                             check=True, capture_output=True, text=True).stdout
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc_summary.json"), "w") as f:
        f.write(summary)
    s = json.loads(summary)
    traffic_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(traffic_path) as f:
            traffic = json.load(f)
    except (OSError, ValueError):
        traffic = {}
    try:
        with open(os.path.join(src, "src_hashes.json")) as f:
            hashes = json.load(f)
    except (OSError, ValueError):
        hashes = {}
    for bench_leg, (leg, kernel) in LEGS.items():
        ks = s["legs"].get(leg)
        if not ks:
            continue
        e = ks.get(kernel)
        if not e or "hbm_bytes_per_launch" not in e:
            continue
        traffic[bench_leg] = {
            "kernel": kernel,
            "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
            "fetch_kib": e.get("FETCH_SIZE"),
            "write_kib": e.get("WRITE_SIZE"),
            "read_factor": e.get("read_factor"),
            "mfma_busy_frac": e.get("mfma_busy_frac"),
            "valu_busy_pct": e.get("VALUBusy"),
            "valu_utilization_pct": e.get("VALUUtilization"),
            "profile": tag,
            # the kernel's sources as they were when the counters ran (pmc_all.sh writes
            # src_hashes.json on the box); bench.with_counters marks a mismatch stale
            "src_hash": hashes.get(kernel) or bench.kernel_source_hash(kernel),
        }
        if e.get("valu_issue_cu_cycles") is not None:
            # issue floor: the mix at the measured per-class peaks (tools/valu_calib.py)
            # spread over 256 CUs, at the clock the launch held (GRBM_GUI_ACTIVE / 8 per
            # wall second, MI355X_MICROARCH.md 'DVFS give-back')
            traffic[bench_leg]["valu_issue_cu_cycles"] = e["valu_issue_cu_cycles"]
            traffic[bench_leg]["valu_issue_cu_cycles_lo"] = e.get("valu_issue_cu_cycles_lo")
            traffic[bench_leg]["valu_mix"] = e.get("valu_mix")
            traffic[bench_leg]["grbm_gui_active"] = e.get("GRBM_GUI_ACTIVE")
    with open(traffic_path, "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    print(f"published {tag}: {len(traffic)} legs in {traffic_path}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
