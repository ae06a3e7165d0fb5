"""Run only bench.py's rank-share legs (one rank's band of the 8-GPU decompositions on
this GPU) and print them as one JSON line:  python3 tools/rank_share.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    print(json.dumps(bench.rank_share_legs(dev)), flush=True)
