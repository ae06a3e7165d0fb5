"""bench.py's strong-scaling legs alone on one GPU (for profiling):
    python tools/scaling_legs.py > out.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
print(json.dumps(bench.scaling_legs(dev, None, 0, 1)))
