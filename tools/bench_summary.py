"""Print the headline and every leg's time from a bench JSON line (the last line of the file)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["value"], "col/s", round(d["ms_per_step"] * 1e3, 2), "us", "frac", round(d["roofline"]["frac"], 3),
      "kernel us", round(d["roofline"].get("mean_launch_us", 0), 2))
for sec in ("extra", "extra_scaling"):
    for k, v in d.get(sec, {}).items():
        if isinstance(v, dict):
            keys = [x for x in ("ms_per_step", "ms_per_call", "frac", "traffic_ratio", "cpu_baseline") if x in v]
            print(f"{k:45s}", {x: (round(v[x], 4) if isinstance(v[x], float) else v[x]) for x in keys
                                if not isinstance(v[x], dict)})
