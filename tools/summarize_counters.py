"""Mean per-dispatch counter values per kernel from rocprofv3 --pmc CSV passes."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+_kernel\w*?)(?:<|\(|I|$)", name)
    return (m.group(1) if m else name)[:48]


def main(root):
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row.get("Kernel_Name", ""))
                if "fv3" not in row.get("Kernel_Name", "") and "kernel" not in k:
                    continue
                vals[(k, row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (k, c), v in sorted(vals.items()):
        print(f"{k:40s} {c:24s} mean {sum(v) / len(v):16.4f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
