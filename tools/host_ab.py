"""Host boundary A/B on the box: wall ms of the pieces of a host call.

rank: one rank's (79, 48, 48) float64 T/q in, float32 dQ1/dQ2 out
  in_pageable    two pageable H2D copies (the runtime's path)
  in_staged_tN   both arrays memcpy'd by N threads into one arena block, one DMA
  out_arena      two D2H DMAs into arena arrays
  call           DenseColumnModel.forward_host (fresh arena outputs)
big: one C384 float64 field (560 MB) in, one float32 field out
  in_pageable, in_staged (PinnedStager with chunk / threads / blocks), out_arena,
  in+out at once (staged in on the stager's stream, DMA out on another)
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import transfer  # noqa: E402


def timeit(fn, n=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e3, 4)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    res = {}
    rng = np.random.default_rng(0)
    # ---- rank call pieces
    T = rng.normal(260, 15, (79, 48, 48))
    q = rng.uniform(0, 0.02, (79, 48, 48))
    dT = torch.empty(T.shape, dtype=torch.float64, device=dev)
    dq = torch.empty_like(dT)
    h = torch.cuda.current_stream().cuda_stream
    res["rank_in_pageable"] = timeit(lambda: (transfer.host_copy(dT, T, h), transfer.host_copy(dq, q, h)))
    blk = transfer.empty_host((2,) + T.shape, np.float64)
    dd = torch.empty((2,) + T.shape, dtype=torch.float64, device=dev)
    import concurrent.futures as cf

    for nt in (1, 2, 4):
        pool = cf.ThreadPoolExecutor(nt) if nt > 1 else None

        def staged():
            if pool is None:
                np.copyto(blk[0], T)
                np.copyto(blk[1], q)
            else:
                parts = [(blk[0], T), (blk[1], q)]
                if nt == 4:
                    parts = [(blk[i][:40], a[:40]) for i, a in enumerate((T, q))] + \
                            [(blk[i][40:], a[40:]) for i, a in enumerate((T, q))]
                list(pool.map(lambda p: np.copyto(*p), parts))
            transfer.host_copy(dd, blk, h)

        res[f"rank_in_staged_t{nt}"] = timeit(staged)
    o1 = torch.empty(T.shape, dtype=torch.float32, device=dev)
    o2 = torch.empty_like(o1)
    out = [transfer.empty_host(T.shape, np.float32) for _ in range(2)]
    res["rank_out_arena"] = timeit(lambda: (transfer.host_copy(out[0], o1, h), transfer.host_copy(out[1], o2, h)))
    plain = [np.empty(T.shape, np.float32) for _ in range(2)]
    res["rank_out_pageable"] = timeit(lambda: (transfer.host_copy(plain[0], o1, h),
                                               transfer.host_copy(plain[1], o2, h)))
    from fv3net_amd import workloads as W

    wl = W.make_dense_workload(48, seed=3, device=dev)
    res["rank_call_forward_host"] = timeit(lambda: wl.model.forward_host([T, q], [0, 0]))
    # ---- one C384 float64 field
    big = rng.normal(size=(6, 79, 384, 384))
    dbig = torch.empty(big.shape, dtype=torch.float64, device=dev)
    res["big_in_pageable"] = timeit(lambda: transfer.host_copy(dbig, big, h), n=5, warm=1)
    for chunk, threads in ((16, 8), (32, 8), (16, 16), (64, 16)):
        st = transfer.PinnedStager(dev, chunk_bytes=chunk << 20, threads=threads)
        res[f"big_in_staged_c{chunk}_t{threads}"] = timeit(lambda: st.h2d(big, out=dbig), n=5, warm=1)
    dout = torch.empty(big.shape, dtype=torch.float32, device=dev)
    hout = transfer.empty_host(big.shape, np.float32)
    res["big_out_arena"] = timeit(lambda: transfer.host_copy(hout, dout, h), n=5, warm=1)
    s2 = torch.cuda.Stream(device=dev)
    st = transfer.stager(dev)

    def both():
        ev = torch.cuda.Event()
        ev.record()
        s2.wait_event(ev)
        transfer.host_copy(hout, dout, s2.cuda_stream)
        st.h2d(big, out=dbig)
        torch.cuda.current_stream().wait_stream(s2)

    res["big_in_staged_plus_out_arena"] = timeit(both, n=5, warm=1)
    res["gb_in"] = big.nbytes / 1e9
    res["gb_out"] = hout.nbytes / 1e9
    print(json.dumps(res))


if __name__ == "__main__":
    main()
