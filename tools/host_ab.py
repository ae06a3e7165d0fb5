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
    from fv3net_amd import dataset as D
    from fv3net_amd.predictor import DenseColumnPredictor

    cfg = wl.model.config
    pred = DenseColumnPredictor(cfg.input_variables, cfg.output_variables, wl.model)
    X = D.Dataset({cfg.input_variables[0]: D.DataArray(T, ["z", "y", "x"]),
                   cfg.input_variables[1]: D.DataArray(q, ["z", "y", "x"])})
    res["rank_call_predictor"] = timeit(lambda: pred.predict(X), n=50)
    import cProfile
    import io
    import pstats

    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        pred.predict(X)
    pr.disable()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(25)
    with open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "rank_call_profile.txt"), "w") as f:
        f.write(buf.getvalue())
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

    def both_pageable():
        ev = torch.cuda.Event()
        ev.record()
        s2.wait_event(ev)
        transfer.host_copy(hout, dout, s2.cuda_stream)
        transfer.host_copy(dbig, big, torch.cuda.current_stream().cuda_stream)
        torch.cuda.current_stream().wait_stream(s2)

    res["big_in_pageable_plus_out_arena"] = timeit(both_pageable, n=5, warm=1)
    from fv3net_amd import _native

    lib = _native.load()

    def both_kernel_out():
        lib.fv3_copy_to_host(hout.ctypes.data, dout.data_ptr(), hout.nbytes, s2.cuda_stream)
        transfer.host_copy(dbig, big, torch.cuda.current_stream().cuda_stream)
        torch.cuda.current_stream().wait_stream(s2)

    res["big_in_pageable_plus_out_kernel"] = timeit(both_kernel_out, n=5, warm=1)
    res["big_out_kernel"] = timeit(lambda: lib.fv3_copy_to_host(hout.ctypes.data, dout.data_ptr(), hout.nbytes, h),
                                   n=5, warm=1)
    stg = transfer.PinnedStager(dev, min_staged=64 << 20)

    def both_staged_kernel_out():
        lib.fv3_copy_to_host(hout.ctypes.data, dout.data_ptr(), hout.nbytes, s2.cuda_stream)
        stg.h2d(big, out=dbig)
        torch.cuda.current_stream().wait_stream(s2)

    res["big_in_staged_plus_out_kernel"] = timeit(both_staged_kernel_out, n=5, warm=1)
    # the C384 host call itself, default path and with the stager / kernel out-copies
    wl2 = W.make_dense_workload(384, seed=3, device=dev)
    T4 = wl2.inputs[0].double().cpu().numpy()
    q4 = wl2.inputs[1].double().cpu().numpy()
    outs = [transfer.empty_host(T4.shape, np.float32) for _ in range(2)]
    res["c384_call_default"] = timeit(lambda: wl2.model.forward_host([T4, q4], [1, 1], out=outs), n=5, warm=1)
    os.environ["FV3_VARIANTS"] = "1"
    os.environ["FV3_D2H_KERNEL"] = "1"
    res["c384_call_kernel_out"] = timeit(lambda: wl2.model.forward_host([T4, q4], [1, 1], out=outs), n=5, warm=1)
    del os.environ["FV3_D2H_KERNEL"]
    # the pipelined call's pieces, re-staged here to find what serialises the two directions
    bufs = [torch.empty(T4.shape, dtype=torch.float64, device=dev) for _ in range(2)]
    dev_out = [torch.empty(T4.shape, dtype=torch.float32, device=dev) for _ in range(2)]
    s_in, s_out = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)

    def pipe(order, compute=True, out_on="s_out"):
        cur = torch.cuda.current_stream()
        pend = None
        for t in range(6):
            for a, b in zip((T4, q4), bufs):
                transfer.host_copy(b[t], a[t], s_in.cuda_stream if order != "cur" else cur.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(s_in)
            cur.wait_event(ev)
            if compute:
                for o in dev_out:
                    o[t].copy_(bufs[0][t])  # a stand-in kernel on the tile
            ev2 = torch.cuda.Event()
            ev2.record(cur)
            so = s_out if out_on == "s_out" else s_in
            so.wait_event(ev2)
            for h_, o in zip(outs, dev_out):
                transfer.host_copy(h_[t], o[t], so.cuda_stream)
        cur.wait_stream(s_out)
        cur.wait_stream(s_in)

    # forward_host's own cached pieces, timed phase by phase
    _, hb, hruns, hstreams = wl2.model._host_call
    hs_out = hstreams[1]

    def fh_pieces(with_out=True, with_compute=True):
        cur = torch.cuda.current_stream()
        hs_out.wait_stream(cur)
        for t in range(6):
            for a, b in zip((T4, q4), hb):
                transfer.host_copy(b[t], a[t], cur.cuda_stream)
            if with_compute:
                o = hruns[t](cur)
            else:
                o = [x[t] for x in dev_out]
            if with_out:
                ev = torch.cuda.Event()
                ev.record(cur)
                hs_out.wait_event(ev)
                for h_, oo in zip(outs, o):
                    transfer.host_copy(h_[t], oo, hs_out.cuda_stream)
        cur.wait_stream(hs_out)

    res["fh_pieces_all"] = timeit(fh_pieces, n=5, warm=1)
    res["fh_pieces_no_out"] = timeit(lambda: fh_pieces(with_out=False), n=5, warm=1)
    res["fh_pieces_no_compute"] = timeit(lambda: fh_pieces(with_compute=False), n=5, warm=1)
    res["pipe_in_s_in_out_s_out"] = timeit(lambda: pipe("s_in"), n=5, warm=1)
    res["pipe_in_cur_out_s_out"] = timeit(lambda: pipe("cur"), n=5, warm=1)
    res["pipe_no_compute"] = timeit(lambda: pipe("s_in", compute=False), n=5, warm=1)
    res["pipe_in_only"] = timeit(lambda: [transfer.host_copy(b[t], a[t], s_in.cuda_stream)
                                          for t in range(6) for a, b in zip((T4, q4), bufs)], n=5, warm=1)
    res["gb_in"] = big.nbytes / 1e9
    res["gb_out"] = hout.nbytes / 1e9
    print(json.dumps(res))


if __name__ == "__main__":
    main()
