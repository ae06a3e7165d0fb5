"""Print the headline and every leg of a bench JSON line (the last line of the file):
the compact driver line (per leg: ms, frac, ratio, tx, valu, pmc, cpu)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("headline", round(d["value"]), "col/s", round(d["ms_per_step"] * 1e3, 2), "us/step", "frac", round(r["frac"], 3),
      "kernel us", round(r.get("mean_launch_us", 0), 2), "traffic", r.get("traffic"), "| line", len(json.dumps(d)),
      "chars")
for sec in ("extra_scaling", "extra"):
    for k, v in d.get(sec, {}).items():
        print(f"{k:40s}", v)
