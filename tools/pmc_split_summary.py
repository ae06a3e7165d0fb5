"""Summary of tools/pmc_split.sh: per-launch counters of the pair remap kernels."""
import collections
import csv
import sys

for ncol in sys.argv[1:] or ["110592", "884736"]:
    for split in ("0", "1"):
        tot = collections.defaultdict(float)
        for p in ("p1", "p2"):
            for r in csv.DictReader(open(f"gpurun_out/pmsp_{ncol}_{split}/{p}/run_counter_collection.csv")):
                if "mappm_ppm_pair" not in r["Kernel_Name"]:
                    continue
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
        d = {k: v / 3 for k, v in tot.items()}
        print(f"{ncol} split {split}: " + ", ".join(f"{k} {v:.4g}" for k, v in sorted(d.items())))
        w = d["SQ_WAVE_CYCLES"]
        print(f"   VALU/wave {d['SQ_INSTS_VALU'] / d['SQ_WAVES']:.0f}  VALU lane-util {d['SQ_THREAD_CYCLES_VALU'] / (64 * d['SQ_ACTIVE_INST_VALU']):.3f}"
              f"  wait_any {d['SQ_WAIT_ANY'] / w:.3f} wait_inst {d['SQ_WAIT_INST_ANY'] / w:.3f} active_valu {d['SQ_ACTIVE_INST_VALU'] / w:.3f}"
              f"  vmem_rd/wave {d['SQ_INSTS_VMEM_RD'] / d['SQ_WAVES']:.0f} branch/wave {d['SQ_INSTS_BRANCH'] / d['SQ_WAVES']:.0f}")
