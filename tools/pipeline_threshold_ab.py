"""forward_host one call vs tile-pipelined (with the copy fence) vs two pipelined halves,
by size: the crossovers that set DenseColumnModel._PIPELINE_MIN_BYTES and the two-group size.  Float64 (6, 79, n, n) T/q in, float32
out (arena), wall ms, interleaved."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import transfer  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402
from fv3net_amd.dense import DenseColumnModel  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    res = {}
    for n in (12, 24, 48, 96, 192):
        wl = W.make_dense_workload(n, seed=3, device=dev)
        T = wl.inputs[0].double().cpu().numpy()
        q = wl.inputs[1].double().cpu().numpy()
        outs = [transfer.empty_host(T.shape, np.float32) for _ in range(2)]
        line = {}
        for rnd in range(3):
            for mode, thr, two in (("one", 1 << 62, "100000"), ("pipe", 0, "100000"), ("two", 1 << 62, "0")):
                DenseColumnModel._PIPELINE_MIN_BYTES = thr
                os.environ["FV3_VARIANTS"] = "1"
                os.environ["FV3_HOST_TWO_GROUPS_MIB"] = two
                reps = max(5, int(2000 / max(n * n / 64, 1)))
                for _ in range(2):
                    wl.model.forward_host([T, q], [1, 1], out=outs)
                ts = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    wl.model.forward_host([T, q], [1, 1], out=outs)
                    ts.append(time.perf_counter() - t0)
                line.setdefault(mode, []).append(round(float(np.median(ts)) * 1e3, 4))
        res[f"C{n}_{2 * T.nbytes >> 20}MiB"] = line
        print(n, json.dumps(line), flush=True)
        del wl
    print(json.dumps(res))


if __name__ == "__main__":
    main()
