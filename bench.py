#!/usr/bin/env python
"""bench.py — fv3net ML-physics hot path on MI355X (driver contract).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one pass of the hot path over one batch: BASELINE config #2, the
column-wise DenseModel predict (fv3fit PureKerasModel.predict -> Keras predict,
pure_keras.py:98-118) of dQ1/dQ2 from T/q on a C48 79-level state, 13,824
columns per GPU, inputs resident in HBM, one fused HIP kernel per step.
Multi-GPU: each rank owns its own C48 state (columns shard with no data-path
collective) -> "scaling": "weak"; value = all ranks' columns / max-over-ranks time.

Rank 0 prints ONE JSON line on stdout (everything else goes to stderr), with
  roofline:     the fused kernel's algorithmic FLOP per launch / its mean launch
                duration (two HIP events on the kernel's own stream bracketing the K
                timed launches) vs the f32 MFMA peak; traffic = HBM bytes per launch
                from the committed rocprofv3 PMC pass (profiles/), or null;
  cpu_baseline: the numpy restatement of the same graph (oracle/dense.py) on the
                host cores, Keras-style batch_size=32 chunks (pure_keras.py:112 calls
                model.predict without batch_size), on a bounded sample (N=1, rank 0);
  extra:        other configs measured on the same GPU (N=1, rank 0).
"""
import argparse
import datetime
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HEADLINE_KERNEL = ("fv3::dense_forward_kernel<2,2,4,2,8,float> (csrc/dense.hip: 8-wave blocks, 32-column tiles, "
                   "f32 inputs)")
METRIC = "grid-columns/s ML-physics step (C48 & C384, 79L); HBM GB/s vs gfx950 peak"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--res", type=int, default=48, help="cubed-sphere resolution per GPU (C48)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extra", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--settle-ms", type=float, default=300.0,
                   help="untimed clock-settle phase before the W warmup steps (see timed_steps)")
    p.add_argument("--legs-out", default=None, help="write the verbose per-leg records (JSON) here")
    p.add_argument("--legs-timeout", type=float, default=480.0, help="seconds allowed for the legs' child process")
    p.add_argument("--legs-only", default=None, help=argparse.SUPPRESS)
    return p.parse_args()


def timed_steps(step, steps, warmup, dist=None, settle_ms=0.0):
    """Clock settle, W untimed steps, then exactly K timed steps bracketed by barrier +
    sync.  Returns (wall seconds, mean seconds per launch).  The launch time comes from
    two HIP events recorded on the stream the kernels run on (torch's current stream,
    which the product passes to every launch) around the K back-to-back launches:
    each step is exactly one kernel, so span / K is its average duration.  Events per
    launch would add ~6 us of queue overhead per step to the wall clock.

    Settle: the same step runs untimed for ``settle_ms`` of wall time first.  The
    MI355X shader clock ramps over ~100 ms of sustained load: a C48 launch measured
    after 20 launches runs at ~2.13 GHz, after 3,000 at ~2.38 GHz (52.9 vs 47.3 us,
    tools/pmc_drive.py), so without it a short K times the ramp, not the kernel."""
    import torch

    # the settle keeps the GPU busy without a gap: the host waits on the event recorded
    # a few batches back (bounding the queue), never on an empty queue, so the clock
    # ramp is not reset by idle gaps every batch.  It runs for at least settle_ms and
    # then until the per-batch time has converged (the last 4 batches of 100 steps within
    # 1 % of each other), at most 10x settle_ms: on a box that was idle before the
    # process started, 300 ms left the first timed launches ~8 % slow (r03f: 46.3 us
    # vs 42.7 us for the same kernel a minute later on the same box)
    t_start = time.perf_counter()
    t_min, t_max = t_start + settle_ms * 1e-3, t_start + 10.0 * settle_ms * 1e-3
    marks, batch_ms = [], []
    prev = None
    while settle_ms > 0:
        now = time.perf_counter()
        if now >= t_max:
            break
        if now >= t_min and len(batch_ms) >= 4:
            last = batch_ms[-4:]
            if max(last) <= 1.01 * min(last):
                break
        if prev is None:
            prev = torch.cuda.Event(enable_timing=True)
            prev.record()
        for _ in range(100):
            step()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((prev, ev))
        prev = ev
        if len(marks) > 4:
            a, b = marks.pop(0)
            b.synchronize()
            batch_ms.append(a.elapsed_time(b))
    for a, b in marks:
        b.synchronize()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return wall, e0.elapsed_time(e1) * 1e-3 / steps


# the translation unit that defines each profiled kernel (csrc/); a PMC record carries the
# hash of that file and every csrc/ header it includes, taken when the counters were
# published (tools/pmc_publish.py), so a record of a kernel changed since is detectable
KERNEL_TU = {
    "dense_forward_kernel": "dense.hip",
    "dense_b3_kernel": "dense_b3.hip",
    "mappm_": "mappm.hip",
    "regrid_coarsen": "coarsen.hip",
    "ml_epilogue": "stepper.hip",
    "area_": "reduce.hip",
    "level_": "reduce.hip",
    "fold_rows": "reduce.hip",
}


def kernel_sources(kernel):
    """csrc/ files the kernel's code depends on: its translation unit and the csrc/
    headers it includes, transitively (the public ABI header is not hashed)."""
    csrc = os.path.join(ROOT, "fv3net_amd", "csrc")
    tu = next((f for k, f in KERNEL_TU.items() if kernel.startswith(k)), None)
    if tu is None:
        return []
    seen, todo = [], [tu]
    fast = tu.replace(".hip", "_fast.hip")  # the fast-arithmetic unit that includes it (mappm_fast.hip)
    if os.path.exists(os.path.join(csrc, fast)):
        todo.append(fast)
    while todo:
        f = todo.pop()
        if f in seen or not os.path.exists(os.path.join(csrc, f)):
            continue
        seen.append(f)
        with open(os.path.join(csrc, f)) as fh:
            for line in fh:
                m = re.match(r'\s*#include\s+"([^"/]+)"', line)
                if m:
                    todo.append(m.group(1))
    return sorted(seen)


def kernel_source_hash(kernel):
    """sha256 (first 16 hex digits) of the kernel's csrc/ sources, or None."""
    files = kernel_sources(kernel)
    if not files:
        return None
    h = hashlib.sha256()
    for f in files:
        h.update(f.encode())
        with open(os.path.join(ROOT, "fv3net_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_record(leg, path=None):
    """The committed PMC record of a bench leg (profiles/pmc_traffic.json, written by
    tools/pmc_all.sh + tools/pmc_publish.py), or {}.  ``stale`` is True when the record
    carries no source hash or one that differs from the tree's sources of its kernel."""
    path = path or os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            r = dict(json.load(f).get(leg, {}))
    except (OSError, ValueError):
        return {}
    if r:
        r["stale"] = r.get("src_hash") is None or r.get("src_hash") != kernel_source_hash(r.get("kernel", ""))
    return r


def pmc_traffic(leg):
    """HBM bytes per launch of the leg's dominant kernel from the committed PMC passes
    (FETCH_SIZE x calibrated read factor + WRITE_SIZE), or None when there is no record
    or the record describes an older version of the kernel's sources."""
    r = pmc_record(leg)
    return None if r.get("stale", True) else r.get("hbm_bytes_per_launch")


def with_counters(leg, rec, alg_bytes=None):
    """Attach the committed counter evidence of ``leg`` to its bench record: HBM traffic
    per launch (and its ratio to the algorithmic bytes), MFMA busy fraction, VALU busy /
    utilisation, and which profile they come from."""
    r = pmc_record(leg)
    if not r:
        rec["traffic"] = None
        return rec
    if r["stale"]:  # counters of an older version of the kernel: reported, never as traffic
        rec["traffic"] = None
        rec["pmc_stale"] = {"profile": r.get("profile"), "hbm_bytes_per_launch": r.get("hbm_bytes_per_launch")}
        return rec
    rec["traffic"] = r.get("hbm_bytes_per_launch")
    if alg_bytes and rec["traffic"]:
        rec["traffic_over_algorithmic"] = rec["traffic"] / alg_bytes
    for k in ("kernel", "mfma_busy_frac", "valu_busy_pct", "valu_utilization_pct"):
        if r.get(k) is not None:
            rec[k if k != "kernel" else "pmc_kernel"] = r[k]
    if r.get("valu_issue_cu_cycles") and r.get("grbm_gui_active"):
        # VALU issue roofline: the launch's instruction mix at the measured per-class
        # issue peaks (tools/valu_calib.py -> profiles/valu_calib.json: 1.68 full-rate,
        # 0.97 half-rate, 0.49 transcendental wave-instructions per CU-cycle) over the
        # CU-cycles the launch took (GRBM_GUI_ACTIVE / 8 XCDs, the same dispatch)
        from fv3net_amd.workloads import N_CU

        cu_cycles = N_CU * r["grbm_gui_active"] / 8
        rec["valu_issue_frac"] = r["valu_issue_cu_cycles"] / cu_cycles
        if r.get("valu_issue_cu_cycles_lo"):  # the unsplit rest (v_mov among it) at full rate
            rec["valu_issue_frac_lo"] = r["valu_issue_cu_cycles_lo"] / cu_cycles
        rec["valu_mix"] = r.get("valu_mix")
    rec["pmc_profile"] = r.get("profile")
    return rec


def cpu_baseline(wl, seconds):
    """Reference-arithmetic CPU restatement (oracle/dense.py) on a bounded sample."""
    from threadpoolctl import threadpool_info

    from oracle.dense import dense_predict

    p = wl.model.oracle_params()
    # one C48 tile of columns, [N, z] sample-major as Keras sees them (pure_keras.py:111)
    T = wl.inputs[0][0].reshape(79, -1).T.contiguous().cpu().numpy()
    q = wl.inputs[1][0].reshape(79, -1).T.contiguous().cpu().numpy()
    n = T.shape[0]
    cols = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for s in range(0, n, 32):  # Keras model.predict default batch_size=32
            dense_predict([T[s:s + 32], q[s:s + 32]], p, np.float32)
        cols += n
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    reps = 0
    while time.perf_counter() - t1 < max(1.0, seconds / 5):
        dense_predict([T, q], p, np.float32)
        reps += 1
    single = reps * n / (time.perf_counter() - t1)
    threads = max([i.get("num_threads", 1) for i in threadpool_info()] + [1])
    return {
        "value": cols / dt,
        "unit": "columns/s",
        "cores": int(threads),
        "kind": "port",
        "sample": f"{cols} columns of one C48 tile ({n} columns/pass) through oracle/dense.py "
                  f"float32 in Keras-default batch_size=32 chunks, {dt:.1f} s; numpy BLAS threads="
                  f"{threads}; single-batch (no Keras chunking) = {single:.3e} columns/s",
    }


def max_over_ranks(x, dist, dev):
    import torch

    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def scaling_legs(dev, dist, rank, world, settle_ms=150.0):
    """Strong-scaling legs run at EVERY world size (all ranks): one global problem
    sharded by row bands of the flattened (tile, y) rows; value = the
    global columns / the max-over-ranks wall time per step.
      stepper_c96_sharded: config #4, the ML-stepper step on a C96 float64 state with
        the per-step exchange of the global-mean / limiter-profile row partials
        (all-gather over RCCL, folded in global row order: the same bits at any N);
      predict_mappm_c384_sharded: north_star's fused predict + mappm at C384 x 79L."""
    import torch

    from fv3net_amd import workloads as W

    out = {}
    wl = W.make_sharded_stepper_workload(96, rank, world, seed=11, device=dev)
    steps = 30
    wall, t = timed_steps(wl.step, steps, 3, dist, settle_ms=settle_ms)
    wall = max_over_ranks(wall, dist, dev)
    del wl
    wl = W.make_sharded_stepper_workload(96, rank, world, seed=11, device=dev)  # fresh state: exactly 1 step
    means, profile = W.ShardedStepperWorkload.means(wl.step())
    out["stepper_c96_sharded"] = {
        "columns_per_s": wl.ncol_global / (wall / steps), "ms_per_step": wall / steps * 1e3,
        "scaling": "strong", "columns_global": wl.ncol_global, "columns_per_rank_max": wl.ncol,
        "global_means": [float(x) for x in means.cpu()],
        "limiter_profile_sum": float(profile.sum().item()),
        "exchange_bytes_per_rank_per_step": wl.exchange_bytes,
        "exchange": "all-gather of 6 float64 row partials per grid row (global means, folded in row order) + "
                    "all-reduce of the 79 integer limiter counts (float64, exact in any order)",
        "note": "wall clock per step incl. the per-step all-gather; global_means / limiter_profile_sum after "
                "one step from the seeded state carry the same bits at any N"}
    del wl
    wl = W.make_predict_mappm_workload(384, rank, world, seed=21, device=dev)
    steps = 10
    wall, t = timed_steps(wl.step, steps, 2, dist, settle_ms=settle_ms)
    wall = max_over_ranks(wall, dist, dev)
    out["predict_mappm_c384_sharded"] = {
        "columns_per_s": wl.ncol_global / (wall / steps), "ms_per_step": wall / steps * 1e3,
        "scaling": "strong", "columns_global": wl.ncol_global, "columns_per_rank_max": wl.ncol,
        "gpu_ms_per_step_rank0": t * 1e3,
        "bytes_per_column_kernels": wl.bytes_per_column,
        "hbm_gbs_per_gpu_kernels": wl.ncol * wl.bytes_per_column / t / 1e9,
        "tflops_per_gpu_dense": wl.ncol * wl.flops_per_column / t / 1e12,
        # committed PMC evidence of the step's two kernels (world-1 profile)
        "kernels": {"dense": with_counters("predict_mappm_c384", {}),
                    "mappm_pair": with_counters("predict_mappm_c384_mappm", {})}}
    del wl
    # the same step with the predict on the bf16x6 kernel (f32-level error, 1e-5 per level)
    wl = W.make_predict_mappm_workload(384, rank, world, seed=21, device=dev, precision="bf16x6")
    wall, t = timed_steps(wl.step, steps, 2, dist, settle_ms=settle_ms)
    wall = max_over_ranks(wall, dist, dev)
    out["predict_mappm_c384_sharded_bf16x6"] = {
        "columns_per_s": wl.ncol_global / (wall / steps), "ms_per_step": wall / steps * 1e3,
        "scaling": "strong", "columns_global": wl.ncol_global, "columns_per_rank_max": wl.ncol,
        "gpu_ms_per_step_rank0": t * 1e3, "precision": "bf16x6",
        "kernels": {"dense": with_counters("predict_mappm_c384_bf16x6", {}),
                    "mappm_pair": with_counters("predict_mappm_c384_mappm", {})}}
    del wl
    torch.cuda.empty_cache()
    return out


def rank_share_legs(dev, settle_ms=150.0, world=8):
    """One rank's share of the 8-GPU target decompositions, run on this one GPU
    (runtime/segmented_run/run.py:34-46 gives every rank its own
    subdomain, runtime/metrics.py:18-32 is the per-step exchange): rank 0's band of the
    flattened (tile, y) rows, each beside the full grid on the same GPU.
    ``ratio_to_full_over_world`` = share time / (full-grid time / world): 1.0 is perfect
    strong scaling of the per-GPU work; above 1 is where the 8-GPU curve flattens (the
    smaller grid fills the 256 CUs less well, or fixed per-launch costs dominate)."""
    import torch

    from fv3net_amd import workloads as W

    def kernel_time(fn, n):
        _, t = timed_steps(fn, n, 3, settle_ms=settle_ms)
        return t

    out = {}
    # config #4: C96 stepper, 6,912 columns per rank at world 8; the exchange (all-gather of
    # the row partials + all-reduce of the limiter counts) stubbed by a local copy
    rec = {}
    for w in (1, world):
        wl = W.make_sharded_stepper_workload(96, 0, w, seed=11, device=dev, stub_exchange=True)
        steps = 30
        wall, _ = timed_steps(wl.step, steps, 3, settle_ms=settle_ms)
        tp = kernel_time(wl.bound, 30)  # the step's predict alone (float64 state read in place)
        rec[w] = {"ncol": wl.ncol, "step_ms": wall / steps * 1e3, "predict_ms": tp * 1e3,
                  "predict_frac_f32_mfma_peak": wl.ncol * wl.model.config.flops_per_column() / tp / 1e12
                  / W.FP32_MFMA_PEAK_TFLOPS, "exchange_bytes": wl.exchange_bytes}
        del wl
    out["stepper_c96_rank_of_8"] = {
        "columns_per_rank": rec[world]["ncol"], "ms_per_step": rec[world]["step_ms"],
        "columns_per_s_per_gpu": rec[world]["ncol"] / (rec[world]["step_ms"] * 1e-3),
        "predict_ms": rec[world]["predict_ms"], "predict_frac_f32_mfma_peak": rec[world]["predict_frac_f32_mfma_peak"],
        "full_grid_ms_per_step": rec[1]["step_ms"], "full_grid_predict_ms": rec[1]["predict_ms"],
        "ratio_to_full_over_world": rec[world]["step_ms"] / (rec[1]["step_ms"] / world),
        "predict_ratio_to_full_over_world": rec[world]["predict_ms"] / (rec[1]["predict_ms"] / world),
        "exchange_bytes_per_rank_per_step": rec[world]["exchange_bytes"],
        "note": "wall clock per step: predict, the fused stepper epilogue, the row partials + limiter counts "
                "(one launch), the stubbed exchange's copy + fold (one launch), all four issued by one launch "
                "plan (workloads.ShardedStepperWorkload._bind); the exchange stubbed by a local copy of the "
                "gathered bytes"}
    # config #5: C384 emulator, 110,592 columns per rank at world 8
    for prec in ("bf16x3", "f32"):
        rec = {}
        for w in (1, world):
            wl = W.make_emulator_workload(384, seed=13, device=dev, precision=prec, world=w)
            t = kernel_time(wl.step, 10)
            tf = wl.ncol * wl.flops_per_column / t / 1e12
            rec[w] = {"ncol": wl.ncol, "ms": t * 1e3,
                      "frac": (3 * tf / W.BF16_MFMA_PEAK_TFLOPS) if prec == "bf16x3" else tf / W.FP32_MFMA_PEAK_TFLOPS}
            del wl
        key = "frac_bf16_mfma_peak" if prec == "bf16x3" else "frac_f32_mfma_peak"
        out[f"emulator_c384_rank_of_8{'' if prec == 'bf16x3' else '_f32'}"] = {
            "columns_per_rank": rec[world]["ncol"], "ms_per_step": rec[world]["ms"], key: rec[world]["frac"],
            "columns_per_s_per_gpu": rec[world]["ncol"] / (rec[world]["ms"] * 1e-3), "precision": prec,
            "full_grid_ms": rec[1]["ms"], f"full_grid_{key}": rec[1]["frac"],
            "ratio_to_full_over_world": rec[world]["ms"] / (rec[1]["ms"] / world)}
    # north_star's predict + mappm at C384 over 8: 110,592 columns per rank
    for prec in ("f32", "bf16x6"):
        rec = {}
        for w in (1, world):
            wl = W.make_predict_mappm_workload(384, 0, w, seed=21, device=dev, precision=prec)
            wl.step()
            t = kernel_time(wl.step, 10)
            td = kernel_time(wl._bound, 10)
            tm = kernel_time(wl._plans, 10)
            tf = wl.ncol * wl.flops_per_column / td / 1e12
            rec[w] = {"ncol": wl.ncol, "ms": t * 1e3, "dense_ms": td * 1e3, "mappm_ms": tm * 1e3,
                      "dense_frac": tf / W.FP32_MFMA_PEAK_TFLOPS if prec == "f32" else 6 * tf / W.BF16_MFMA_PEAK_TFLOPS}
            del wl
        key = "dense_frac_f32_mfma_peak" if prec == "f32" else "dense_frac_bf16_mfma_peak"
        out[f"predict_mappm_c384_rank_of_8{'' if prec == 'f32' else '_bf16x6'}"] = {
            "columns_per_rank": rec[world]["ncol"], "ms_per_step": rec[world]["ms"],
            "columns_per_s_per_gpu": rec[world]["ncol"] / (rec[world]["ms"] * 1e-3), "precision": prec,
            "dense_ms": rec[world]["dense_ms"], "mappm_ms": rec[world]["mappm_ms"], key: rec[world]["dense_frac"],
            "full_grid_ms": rec[1]["ms"], "full_grid_dense_ms": rec[1]["dense_ms"],
            "full_grid_mappm_ms": rec[1]["mappm_ms"],
            "ratio_to_full_over_world": rec[world]["ms"] / (rec[1]["ms"] / world),
            "dense_ratio_to_full_over_world": rec[world]["dense_ms"] / (rec[1]["dense_ms"] / world),
            "mappm_ratio_to_full_over_world": rec[world]["mappm_ms"] / (rec[1]["mappm_ms"] / world)}
    for k in out:
        out[k] = with_counters(k, out[k])
    torch.cuda.empty_cache()
    return out


def host_to_host(dev, res, steps=10):
    """The reference's boundary crossing: float64 host (numpy) T/q in, H2D as pageable
    copies or through the library's staging blocks (fv3net_amd/transfer.py), the fused
    predict reading float64 in place, float32 dQ1/dQ2 DMA'd back into the library's
    page-locked arena arrays (pure_keras.py:98-118 runs on host arrays).  Wall time per
    step."""
    import torch

    from fv3net_amd import transfer
    from fv3net_amd import workloads as W

    wl = W.make_dense_workload(res, seed=3, device=dev)
    T = wl.inputs[0].double().cpu().numpy()
    q = wl.inputs[1].double().cpu().numpy()
    host_out = [transfer.empty_host(T.shape, np.float32), transfer.empty_host(T.shape, np.float32)]

    def step():  # the product's host boundary (the predictor's numpy path), outputs reused
        wl.model.forward_host([T, q], [1, 1], out=host_out)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    wall = (time.perf_counter() - t0) / steps
    nbytes = T.nbytes + q.nbytes + sum(h.nbytes for h in host_out)
    return {"columns_per_s": wl.ncol / wall, "ms_per_step": wall * 1e3, "host_bytes_per_step": nbytes,
            "pcie_inclusive_gbs": nbytes / wall / 1e9,
            "host_path": transfer.host_path(),
            "note": "float64 numpy in -> DenseColumnModel.forward_host: H2D (see host_path), the fused predict "
                    "(f64 read in place), D2H into float32 numpy outputs reused across calls (library arena "
                    "when host_path is arena); tile blocks pipelined over two streams from 128 MiB (C384), two halves from 48 MiB"}


def predict_mappm_host_to_host(dev, res=384, steps=5, bands=6, fence=True):
    """north_star's predict + mappm with the host boundary included: float64 numpy T/q
    (z, rows, x) and float32 numpy edge pressures pe1/pe2 (z+1, columns; f2py hands the
    reference's mappm float32 arrays) in, the fused predict reading float64 in place, the
    two-field mappm of both tendencies, and the float32 remapped tendencies back to numpy.
    The caller's inputs cross as pageable pitched copies (caller memory is never
    page-locked), the outputs live in the library's page-locked arena (reused across
    calls), and the columns run in ``bands`` bands pipelined over two streams: band b + 1's
    pitched in-copies (``transfer.copy_band``) and band b's out-copies overlap.  Wall time
    per step."""
    import torch

    from fv3net_amd import transfer
    from fv3net_amd import workloads as W
    from fv3net_amd.mappm import MappmMultiPlan

    wl = W.make_predict_mappm_workload(res, seed=21, device=dev)
    T = wl.inputs[0].double().cpu().numpy()
    q = wl.inputs[1].double().cpu().numpy()
    pe1 = wl.pe1.cpu().numpy()
    pe2 = wl.pe2.cpu().numpy()
    nz, ncol = T.shape[0], wl.ncol
    T2, q2 = T.reshape(nz, ncol), q.reshape(nz, ncol)
    dT = torch.empty((nz, ncol), dtype=torch.float64, device=dev)
    dq = torch.empty((nz, ncol), dtype=torch.float64, device=dev)
    d1 = torch.empty_like(wl.pe1)
    d2 = torch.empty_like(wl.pe2)
    outs = [o.view(nz, ncol) for o in wl.outputs]
    host_out = [transfer.empty_host(tuple(r.shape), np.float32) for r in wl.remapped]
    # band edges on whole grid rows
    rows = ncol // res
    edges = [res * (rows * b // bands) for b in range(bands + 1)]
    runs = []
    for b in range(bands):
        c0, c1 = edges[b], edges[b + 1]
        bound = wl.model.bind([dT[:, c0:c1], dq[:, c0:c1]], level_axes=[0, 0],
                              outputs=[o[:, c0:c1] for o in outs], out_level_axis=0)
        plan = MappmMultiPlan(d1[:, c0:c1], [o[:, c0:c1] for o in outs], d2[:, c0:c1], 1, 1,
                              out=[r[:, c0:c1] for r in wl.remapped])
        runs.append((c0, c1, bound, plan))
    s_out = torch.cuda.Stream(device=dev)
    s_idle = torch.cuda.Stream(device=dev)  # transfer.copy_fence

    def step():
        cur = torch.cuda.current_stream()
        for c0, c1, bound, plan in runs:
            # band b's in-copies (pitched, the runtime's pageable path, on the compute
            # stream: the host waits for them while band b - 1's out-copies run on s_out)
            for h, d in ((T2, dT), (q2, dq), (pe1, d1), (pe2, d2)):
                transfer.copy_band(d[:, c0:c1], h[:, c0:c1], cur.cuda_stream)
            if fence:
                transfer.copy_fence(cur, s_idle)
            bound(cur)
            plan()
            for h, r in zip(host_out, wl.remapped):  # arena outputs: asynchronous DMA
                transfer.copy_band(h[:, c0:c1], r[:, c0:c1], s_out)
        cur.wait_stream(s_out)
        cur.synchronize()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    wall = (time.perf_counter() - t0) / steps
    nbytes = T.nbytes + q.nbytes + pe1.nbytes + pe2.nbytes + sum(h.nbytes for h in host_out)
    # the same state device-resident (float32 inputs: the f64 host values are their exact
    # widening) must give the same bits
    wl.step()
    wl.step()
    same = all(np.array_equal(h.view(np.uint32), r.cpu().numpy().view(np.uint32))
               for h, r in zip(host_out, wl.remapped))
    return {"columns_per_s": wl.ncol / wall, "ms_per_step": wall * 1e3, "host_bytes_per_step": nbytes,
            "pcie_inclusive_gbs": nbytes / wall / 1e9, "bit_identical_to_device_resident": bool(same),
            "bands": bands,
            "host_path": transfer.host_path(),
            "note": "float64 numpy T/q + float32 numpy pe1/pe2 in (see host_path) -> per column band: "
                    "pitched H2D, fused predict (f64 read in place), two-field mappm of dQ1/dQ2 (kord 1, iv 1), "
                    "pitched D2H into float32 numpy; bands pipelined over two streams"}


def rank_call_host_to_host(dev, calls=30):
    """The reference's real per-rank call: one rank's C48 subdomain,
    (79, 48, 48) float64 host arrays of T / q in a Dataset, through the drop-in
    ``DenseColumnPredictor.predict`` (pure_keras.py:98-118 boundary): host -> device,
    the fused predict, float32 (79, 48, 48) numpy outputs back.  Wall time per call."""
    from fv3net_amd import dataset as D
    from fv3net_amd import transfer
    from fv3net_amd import workloads as W
    from fv3net_amd.predictor import DenseColumnPredictor

    wl = W.make_dense_workload(48, seed=3, device=dev)
    cfg = wl.model.config
    pred = DenseColumnPredictor(cfg.input_variables, cfg.output_variables, wl.model)
    T = wl.inputs[0][0].double().cpu().numpy()  # tile 0: (z, y, x)
    q = wl.inputs[1][0].double().cpu().numpy()
    X = D.Dataset({cfg.input_variables[0]: D.DataArray(T, ["z", "y", "x"]),
                   cfg.input_variables[1]: D.DataArray(q, ["z", "y", "x"])})
    for _ in range(3):
        out = pred.predict(X)
    t0 = time.perf_counter()
    for _ in range(calls):
        out = pred.predict(X)
    wall = (time.perf_counter() - t0) / calls
    assert out[cfg.output_variables[0]].values.dtype == np.float32
    ncol = T.shape[1] * T.shape[2]
    return {"columns_per_s": ncol / wall, "ms_per_call": wall * 1e3, "columns_per_call": ncol,
            "host_bytes_per_call": T.nbytes + q.nbytes + 2 * ncol * 79 * 4,
            "host_path": transfer.host_path(),
            "note": "one rank's (79,48,48) float64 numpy T/q Dataset -> DenseColumnPredictor.predict -> float32 "
                    "(79,48,48) numpy dQ1/dQ2 Dataset, fresh outputs each call (the drop-in call, host boundary "
                    "included)"}


def _ref_mappm_worker(args):
    from oracle import mappm as OM

    pe1, q, pe2, seconds = args
    cols, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        OM.reference_mappm(pe1, q, pe2, 1, 1)
        cols += pe1.shape[1]
    return cols, time.perf_counter() - t0


def reference_mappm_cpu_procs(procs=8, seconds=5.0):
    """the reference mappm.f90 (flang, oracle/_ref) in ``procs``
    single-threaded processes at once, each on its own config #3 columns: aggregate
    columns/s."""
    import multiprocessing as mp

    from oracle import mappm as OM

    if not OM.reference_available():
        return None
    rng = np.random.default_rng(1)
    n = 4096
    base = np.linspace(200.0, 1800.0, 79)[:, None]
    jobs = []
    for _ in range(procs):
        delp = (base * rng.uniform(0.99, 1.01, (79, n))).astype(np.float32)
        pe1 = np.concatenate([np.full((1, n), 300.0, np.float32), 300.0 + np.cumsum(delp, 0, dtype=np.float32)])
        d2 = (base * rng.uniform(0.99, 1.01, (79, n))).astype(np.float32)
        pe2 = np.concatenate([np.full((1, n), 300.0, np.float32), 300.0 + np.cumsum(d2, 0, dtype=np.float32)])
        q = rng.normal(250.0, 10.0, (79, n)).astype(np.float32)
        jobs.append((pe1, q, pe2, seconds))
    # close + join (not the context manager's terminate()): the workers finish their own
    # interpreter shutdown, so no SIGTERM lands in a finalising worker (a profiler run
    # would log those as "Aborted")
    pool = mp.get_context("spawn").Pool(procs)
    try:
        res = pool.map(_ref_mappm_worker, jobs)
        pool.close()
    except BaseException:
        pool.terminate()
        raise
    finally:
        pool.join()
    cols = sum(c for c, _ in res)
    dt = max(t for _, t in res)
    return {"value": cols / dt, "unit": "columns/s", "cores": procs, "kind": "reference",
            "sample": f"{procs} processes x {seconds:.0f} s, each its own 4096 config #3 columns (79 -> 79, kord 1) "
                      f"through the reference mappm.f90 (flang -O2, oracle/_ref) in 512-column chunks"}


def coarsen_cpu_baseline(seconds=10.0):
    """Config #3's coarsen on the host: oracle/coarsen.py (numpy + the C restatement of
    mappm.f90, the reference's regrid_to_area_weighted_pressure -> weighted_block_average
    arithmetic) on a bounded slab of a C384 tile, one field, f = 8: fine columns/s."""
    from oracle import coarsen as OC

    rng = np.random.default_rng(2)
    ny, nx = 64, 384
    base = np.linspace(200.0, 1800.0, 79)[None, :, None, None]
    delp = (base * rng.uniform(0.99, 1.01, (1, 79, ny, nx))).astype(np.float32)
    area = rng.uniform(0.5, 1.0, (1, ny, nx)).astype(np.float32)
    T = rng.normal(250.0, 10.0, (1, 79, ny, nx)).astype(np.float32)
    cols, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        OC.coarsen_on_pressure(delp, area, [T], 8)
        cols += ny * nx
    dt = time.perf_counter() - t0
    return {"value": cols / dt, "unit": "fine columns/s", "cores": 1, "kind": "port",
            "sample": f"{cols} fine columns ({ny}x{nx} slabs of a C384 tile, 79 levels, 1 field, f = 8) through "
                      f"oracle/coarsen.py (numpy + the C restatement of mappm.f90), {dt:.1f} s, 1 core"}


def _blas_threads():
    from threadpoolctl import threadpool_info

    return int(max([i.get("num_threads", 1) for i in threadpool_info()] + [1]))


def stepper_cpu_baseline(wl, seconds=10.0):
    """Config #4's step on the host: the numpy restatement of the predict (oracle/dense.py,
    float32, Keras-default batch_size=32 chunks as PureKerasModel.predict runs it,
    pure_keras.py:112) then oracle/stepper.py's limiter / diagnostics / apply epilogue
    (the reference's numpy arithmetic, machine_learning.py:239-309) on one C96 tile of the
    same float64 state: columns/s."""
    from oracle import stepper as OS
    from oracle.dense import dense_predict

    p = wl.model.oracle_params()
    st = {k: v[0].reshape(v.shape[1], -1).cpu().numpy() if v.dim() == 4 else v[0].reshape(-1).cpu().numpy()
          for k, v in wl.state.items()}
    T, q = st["air_temperature"], st["specific_humidity"]
    delp, precip = st["pressure_thickness_of_atmospheric_layer"], st["total_precipitation"]
    Ts, qs = T.T.astype(np.float32), q.T.astype(np.float32)
    n = Ts.shape[0]
    cols, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        outs = [dense_predict([Ts[s:s + 32], qs[s:s + 32]], p, np.float32) for s in range(0, n, 32)]
        dq1 = np.concatenate([o[0] for o in outs]).T
        dq2 = np.concatenate([o[1] for o in outs]).T
        OS.epilogue(dq1, dq2, q, delp, T, precip, wl.dt)
        cols += n
    dt = time.perf_counter() - t0
    threads = _blas_threads()
    return {"value": cols / dt, "unit": "columns/s", "cores": threads, "kind": "port",
            "sample": f"{cols} columns of one C96 tile ({n}/pass): oracle/dense.py float32 predict in batch_size=32 "
                      f"chunks + oracle/stepper.py epilogue on the float64 state, {dt:.1f} s; numpy BLAS "
                      f"threads={threads}"}


def emulator_cpu_baseline(wl, seconds=10.0, ncol=16384, batch=1024):
    """Config #5 on the host: oracle/emulator.py's forward (the emulator's numpy
    restatement, float32) over ``ncol`` columns of the same C384 state in the reference's
    batch_size=1024 chunks (external/emulation/emulation/models.py:20): columns/s."""
    from oracle import emulator as OE

    raw = {k: v[:, :ncol].T.contiguous().cpu().numpy() for k, v in wl.state.items()}
    params = wl.emulator.params_by_name()
    spec = OE.zhao_carr_spec()
    cols, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for s in range(0, ncol, batch):
            OE.forward({k: v[s:s + batch] for k, v in raw.items()}, spec, params, np.float32)
        cols += ncol
    dt = time.perf_counter() - t0
    threads = _blas_threads()
    return {"value": cols / dt, "unit": "columns/s", "cores": threads, "kind": "port",
            "sample": f"{cols} columns ({ncol} of the C384 state per pass) through oracle/emulator.py float32 in "
                      f"batch_size={batch} chunks, {dt:.1f} s; numpy BLAS threads={threads}"}


def reference_mappm_cpu(seconds=5.0):
    """The reference's own Fortran mappm (flang build in oracle/_ref)
    timed on one host core in 512-column chunks on config #3 columns (79 -> 79, kord 1).
    A reported baseline only."""
    from oracle import mappm as OM

    if not OM.reference_available():
        return None
    rng = np.random.default_rng(0)
    n = 8192
    base = np.linspace(200.0, 1800.0, 79)[:, None]
    delp = (base * rng.uniform(0.99, 1.01, (79, n))).astype(np.float32)
    pe1 = np.concatenate([np.full((1, n), 300.0, np.float32), 300.0 + np.cumsum(delp, 0, dtype=np.float32)])
    d2 = (base * rng.uniform(0.99, 1.01, (79, n))).astype(np.float32)
    pe2 = np.concatenate([np.full((1, n), 300.0, np.float32), 300.0 + np.cumsum(d2, 0, dtype=np.float32)])
    q = rng.normal(250.0, 10.0, (79, n)).astype(np.float32)
    cols = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        OM.reference_mappm(pe1, q, pe2, 1, 1)
        cols += n
    dt = time.perf_counter() - t0
    return {"value": cols / dt, "unit": "columns/s", "cores": 1, "kind": "reference",
            "sample": f"{cols} config #3 columns (79 -> 79, kord 1, iv 1) through the reference mappm.f90 "
                      f"(flang -O2, oracle/_ref) in 512-column chunks via ctypes, {dt:.1f} s, 1 core"}


def extra_measurements(dev, settle_ms=150.0, out=None):
    import torch

    from fv3net_amd import workloads as W

    out = {} if out is None else out
    # config #2 at C384 (one GPU, 884,736 columns): MFMA-bound predict
    wl = W.make_dense_workload(384, seed=3, device=dev)
    wall, t = timed_steps(wl.step, 10, 3, settle_ms=settle_ms)
    out["dense_c384"] = with_counters("dense_c384", {
        "columns_per_s": wl.ncol / t, "ms_per_step": t * 1e3,
        "tflops": wl.ncol * wl.flops_per_column / t / 1e12,
        "frac_f32_mfma_peak": wl.ncol * wl.flops_per_column / t / 1e12 / W.FP32_MFMA_PEAK_TFLOPS,
    }, wl.ncol * wl.bytes_per_column)
    del wl
    # mappm: config #3 fine columns (C384 79->79) and config #1 (C12 79->50)
    # the default (tolerance-contract) arithmetic, and the bit-exact one beside it (_exact)
    for name, ncol, kn, kord, exact in (("mappm_c384_79to79_kord1", W.c_columns(384), 79, 1, False),
                                        ("mappm_c384_79to79_kord1_exact", W.c_columns(384), 79, 1, True),
                                        ("mappm_c384_79to79_kord10", W.c_columns(384), 79, 10, False),
                                        ("mappm_c384_79to79_kord10_exact", W.c_columns(384), 79, 10, True),
                                        ("mappm_c12_79to50_kord1", W.c_columns(12), 50, 1, False)):
        wl = W.make_mappm_workload(ncol, 79, kn, kord, seed=5, device=dev, exact=exact)
        wall, t = timed_steps(wl.step, 10, 3, settle_ms=settle_ms)
        gbs = wl.bytes_per_column * ncol / t / 1e9
        out[name] = with_counters(name, {"columns_per_s": ncol / t, "ms_per_step": t * 1e3, "hbm_gbs": gbs,
                                         "frac_hbm_peak": gbs / W.HBM_PEAK_GBS}, wl.bytes_per_column * ncol)
        del wl
    try:
        out["mappm_c384_79to79_kord1"] = dict(out["mappm_c384_79to79_kord1"], cpu_baseline=reference_mappm_cpu(),
                                              cpu_baseline_8proc=reference_mappm_cpu_procs())
    except Exception as e:  # a report, never fatal
        log("reference mappm cpu baseline failed:", repr(e))
    # config #4: one ML-stepper step (predict + fused limiter/diagnostics/apply + global
    # means) on a float64 C96 state, one GPU
    wl = W.make_stepper_workload(96, seed=11, device=dev)
    wall, t = timed_steps(wl.step, 20, 3, settle_ms=settle_ms)
    out["stepper_c96"] = with_counters("stepper_c96", {
        "columns_per_s": wl.ncol / (wall / 20), "ms_per_step": wall / 20 * 1e3,
        "note": "wall clock per step (predict, fused epilogue, area partials: three C-ABI calls marshalled once, "
                "workloads.StepperWorkload._bind); counters: the fused epilogue kernel"})
    try:
        out["stepper_c96"] = dict(out["stepper_c96"], cpu_baseline=stepper_cpu_baseline(wl))
    except Exception as e:  # a report, never fatal
        log("stepper cpu baseline failed:", repr(e))
    del wl
    # the same step with the predict on the bf16x6 split kernel (1e-5 per level like the
    # f32 kernel); the float64 state is cast into bound float32 buffers each step
    wl = W.make_stepper_workload(96, seed=11, device=dev, precision="bf16x6")
    wall, t = timed_steps(wl.step, 20, 3, settle_ms=settle_ms)
    out["stepper_c96_bf16x6"] = {
        "columns_per_s": wl.ncol / (wall / 20), "ms_per_step": wall / 20 * 1e3, "precision": "bf16x6",
        "note": "wall clock per step; predict on dense_b3_kernel<16,2,3,8> after two float64->float32 casts"}
    del wl
    # config #5: Zhao-Carr microphysics emulator on a C384 state.  Its arithmetic is bf16
    # MFMA (1e-3 rel): the bf16x3 kernel (csrc/dense_b3.hip, 3 bf16 MFMAs per f32
    # product, so the bf16 roofline is priced at 3x the algorithmic FLOP); the exact-f32
    # kernel beside it for comparison
    for prec in ("bf16x3", "bf16x6", "f32"):
        wl = W.make_emulator_workload(384, seed=13, device=dev, precision=prec)
        wall, t = timed_steps(wl.step, 10, 3, settle_ms=settle_ms)
        tf = wl.ncol * wl.flops_per_column / t / 1e12
        rec = {"columns_per_s": wl.ncol / t, "ms_per_step": t * 1e3, "precision": prec,
               "tflops_f32_equiv": tf, "hbm_gbs": wl.ncol * wl.bytes_per_column / t / 1e9}
        if prec == "f32":
            rec["frac_f32_mfma_peak"] = tf / W.FP32_MFMA_PEAK_TFLOPS
        else:
            rec["frac_bf16_mfma_peak"] = (3 if prec == "bf16x3" else 6) * tf / W.BF16_MFMA_PEAK_TFLOPS
        leg = {"bf16x3": "emulator_c384", "bf16x6": "emulator_c384_bf16x6", "f32": "emulator_c384_f32"}[prec]
        out[leg] = with_counters(leg, rec, wl.ncol * wl.bytes_per_column)
        if prec == "bf16x3":
            try:
                out[leg] = dict(out[leg], cpu_baseline=emulator_cpu_baseline(wl))
            except Exception as e:  # a report, never fatal
                log("emulator cpu baseline failed:", repr(e))
        del wl
    # config #2's model on the bf16x3 kernel (8e-6 rel: not the headline's exact-f32 path)
    wl = W.make_dense_workload(384, seed=3, device=dev, precision="bf16x3")
    wall, t = timed_steps(wl.step, 10, 3, settle_ms=settle_ms)
    tf = wl.ncol * wl.flops_per_column / t / 1e12
    out["dense_c384_bf16x3"] = with_counters("dense_c384_bf16x3", {
        "columns_per_s": wl.ncol / t, "ms_per_step": t * 1e3, "tflops_f32_equiv": tf,
        "frac_bf16_mfma_peak": 3 * tf / W.BF16_MFMA_PEAK_TFLOPS}, wl.ncol * wl.bytes_per_column)
    del wl
    # config #2's model on the bf16x6 kernel (three bf16 parts per operand, six MFMAs per
    # f32 product: held to the exact-f32 kernel's 1e-5 per-level bound), C48 and C384
    for res, n in ((48, 200), (384, 10)):
        wl = W.make_dense_workload(res, seed=3, device=dev, precision="bf16x6")
        wall, t = timed_steps(wl.step, n, 3, settle_ms=settle_ms)
        tf = wl.ncol * wl.flops_per_column / t / 1e12
        leg = f"dense_c{res}_bf16x6"
        out[leg] = with_counters(leg, {
            "columns_per_s": wl.ncol / t, "ms_per_step": t * 1e3, "tflops_f32_equiv": tf,
            "frac_bf16_mfma_peak": 6 * tf / W.BF16_MFMA_PEAK_TFLOPS,
            "tflops_f32_equiv_over_f32_peak": tf / W.FP32_MFMA_PEAK_TFLOPS}, wl.ncol * wl.bytes_per_column)
        del wl
    # config #3: fused C384 -> C48 pressure-level coarsen (1 and 4 fields), fine columns/s
    for nf, exact in ((1, False), (4, False), (1, True), (4, True)):
        wl = W.make_coarsen_workload(384, 8, nf, seed=7, device=dev, exact=exact)
        wall, t = timed_steps(wl.step, 10, 3, settle_ms=settle_ms)
        gbs = wl.bytes_per_column * wl.ncol_fine / t / 1e9
        leg = f"coarsen_c384_to_c48_{nf}field" + ("_exact" if exact else "")
        out[leg] = with_counters(leg, {
            "fine_columns_per_s": wl.ncol_fine / t, "ms_per_step": t * 1e3, "hbm_gbs": gbs,
            "frac_hbm_peak": gbs / W.HBM_PEAK_GBS}, wl.bytes_per_column * wl.ncol_fine)
        del wl
    try:
        out["coarsen_c384_to_c48_1field"] = dict(out["coarsen_c384_to_c48_1field"],
                                                 cpu_baseline=coarsen_cpu_baseline())
    except Exception as e:  # a report, never fatal
        log("coarsen cpu baseline failed:", repr(e))
    # host -> host (numpy float64 in, numpy float32 out) beside the device-resident legs
    for res in (48, 384):
        out[f"dense_c{res}_host_to_host"] = host_to_host(dev, res)
    out["dense_c48_rank_call_host_to_host"] = rank_call_host_to_host(dev)
    out["predict_mappm_c384_host_to_host"] = predict_mappm_host_to_host(dev)
    torch.cuda.empty_cache()
    for k, v in rank_share_legs(dev, settle_ms).items():
        out[k] = v
    return out


LINE_BUDGET = 7500  # characters of the final stdout line (the driver keeps ~8 KB of stdout)


class LegRecorder(dict):
    """The legs' records as they are produced: every assignment is also written as one
    JSON line to ``path`` (and a ``BENCH_LEG`` line on stderr), so the parent keeps every
    leg that finished even if a later one takes the child process down."""

    def __init__(self, path):
        super().__init__()
        self.path = path

    def __setitem__(self, key, value):
        super().__setitem__(key, value)
        self.emit(key, value)

    def emit(self, key, value):
        line = json.dumps({key: value})
        with open(self.path, "a") as f:
            f.write(line + "\n")
        log("BENCH_LEG", line)


def _sig(x, n=4):
    if isinstance(x, bool) or not isinstance(x, (int, float)):
        return x
    return float(f"{x:.{n}g}")


def compact_leg(rec):
    """One leg's record reduced to what the driver line carries: ms, the roofline
    fraction, the rank-share ratio, traffic over algorithmic bytes, VALU issue fraction,
    the CPU baseline's value, and whether the counters are fresh."""
    if not isinstance(rec, dict):
        return rec
    out = {}
    for k in ("ms_per_step", "ms_per_call"):
        if rec.get(k) is not None:
            out["ms"] = _sig(rec[k])
            break
    for k in ("columns_per_s", "fine_columns_per_s", "columns_per_s_per_gpu"):
        if rec.get(k) is not None:
            out["cps"] = _sig(rec[k], 3)
            break
    frac = [k for k in rec if k.startswith("frac_") or k.startswith("dense_frac_") or k.startswith("predict_frac_")]
    if frac:
        out["frac"] = _sig(rec[frac[0]], 3)
    for src, dst in (("ratio_to_full_over_world", "ratio"), ("dense_ratio_to_full_over_world", "dense_ratio"),
                     ("mappm_ratio_to_full_over_world", "mappm_ratio"), ("traffic_over_algorithmic", "tx"),
                     ("valu_issue_frac", "valu"), ("max_rel_err", "err"), ("bit_identical_to_device_resident", "same")):
        if rec.get(src) is not None:
            out[dst] = _sig(rec[src], 3)
    if rec.get("pmc_profile"):
        out["pmc"] = rec["pmc_profile"]
    if rec.get("pmc_stale"):
        out["pmc"] = f"{rec['pmc_stale'].get('profile')} (stale)"
    for k in ("cpu_baseline", "cpu_baseline_8proc"):
        if isinstance(rec.get(k), dict):
            out["cpu" if k == "cpu_baseline" else "cpu8"] = _sig(rec[k]["value"], 3)
    if isinstance(rec.get("kernels"), dict):
        for name, kr in rec["kernels"].items():
            if isinstance(kr, dict) and kr.get("traffic"):
                out[f"{name}_traffic"] = _sig(kr["traffic"], 3)
    return out


def compact_line(result):
    """The driver's line: the contract fields, roofline, cpu_baseline and a terse
    summary of every leg (the verbose records go to stderr / --legs-out)."""
    line = {k: v for k, v in result.items() if k not in ("extra", "extra_scaling")}
    for sec in ("extra_scaling", "extra"):
        if isinstance(result.get(sec), dict):
            line[sec] = {k: compact_leg(v) for k, v in result[sec].items()}
        elif result.get(sec) is not None:
            line[sec] = result[sec]
    return json.dumps(line)


def run_legs_child(args, timeout):
    """The world-1 legs (extra_scaling + extra) in a child process: a sticky GPU fault or
    a hang in any of them cannot take the headline with it.  Returns (scaling, extra)."""
    fd, path = tempfile.mkstemp(prefix="bench_legs_", suffix=".jsonl")
    os.close(fd)
    cmd = [sys.executable, os.path.abspath(__file__), "--legs-only", path, "--settle-ms", str(args.settle_ms)]
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    status = None
    try:
        p = subprocess.run(cmd, stdout=sys.stderr, stderr=sys.stderr, timeout=timeout, env=env)
        if p.returncode != 0:
            status = f"legs child exited with {p.returncode}"
    except subprocess.TimeoutExpired:
        status = f"legs child killed after {timeout} s"
    legs = {}
    try:
        with open(path) as f:
            for ln in f:
                legs.update(json.loads(ln))
    except (OSError, ValueError) as e:
        status = (status or "") + f"; legs file unreadable: {e!r}"
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass
    scaling = {k[len("scaling/"):]: v for k, v in legs.items() if k.startswith("scaling/")}
    extra = {k: v for k, v in legs.items() if not k.startswith("scaling/")}
    if status:
        log(status)
        extra["_status"] = status
    return scaling, extra


def legs_only(args):
    """Child mode: run every world-1 leg, recording each as it finishes."""
    import torch

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    rec = LegRecorder(args.legs_only)
    settle = min(args.settle_ms, 150.0)
    try:
        for k, v in scaling_legs(dev, None, 0, 1, settle_ms=settle).items():
            rec["scaling/" + k] = v
    except Exception as e:
        log("scaling legs failed:", repr(e))
    extra_measurements(dev, settle_ms=settle, out=rec)


def main():
    args = parse()
    if args.legs_only:
        return legs_only(args)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as tdist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # a rank that fails outside a collective ends the job in minutes, not at the
        # default 10-minute watchdog
        tdist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev,
                                 timeout=datetime.timedelta(minutes=5))
        dist = tdist

    from fv3net_amd import workloads as W

    wl = W.make_dense_workload(args.res, seed=1000 + rank, device=dev)
    wall, kmean = timed_steps(wl.step, args.steps, args.warmup, dist, settle_ms=args.settle_ms)
    if dist is not None:
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    total_cols = wl.ncol * world * args.steps
    value = total_cols / wall
    flops_launch = wl.ncol * wl.flops_per_column
    achieved = flops_launch / kmean / 1e12
    pmc = pmc_record("dense_c48")

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "columns/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_ms": args.settle_ms,
        "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (T~N(260,15) K, q~U(0,0.02); random Glorot weights, norms fitted on the sample)",
        "config": {
            "workload": "config #2: fv3fit DenseModel (2x256) column-wise predict of dQ1/dQ2 from T/q, "
                        f"C{args.res} 79L per GPU, fused normalize->MLP->denormalize kernel",
            "columns_per_gpu": wl.ncol,
            "levels": 79,
            "global_batch": wl.ncol * world,
            "parallelism": f"columns sharded, 1 process/GPU x {world}",
        },
        "roofline": {
            "kernel": HEADLINE_KERNEL,
            "bound": "mfma",
            "achieved": achieved,
            "peak": W.FP32_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / W.FP32_MFMA_PEAK_TFLOPS,
            "traffic": pmc_traffic("dense_c48"),
            "traffic_profile": pmc.get("profile") if not pmc.get("stale", True) else None,
            "algorithmic_flop_per_launch": flops_launch,
            "algorithmic_bytes_per_launch": wl.ncol * wl.bytes_per_column,
            "mean_launch_us": kmean * 1e6,
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(wl, args.cpu_seconds)
        except Exception as e:  # the baseline is a report, never fatal
            log("cpu_baseline failed:", repr(e))
    del wl
    torch.cuda.empty_cache()
    if rank == 0:  # the headline alone, on stderr, before any leg runs
        log("BENCH_HEADLINE", compact_line(result))
    if not args.no_extra:
        if world == 1:
            result["extra_scaling"], result["extra"] = run_legs_child(args, args.legs_timeout)
        else:
            try:  # every rank takes part: one global problem sharded over the ranks
                result["extra_scaling"] = scaling_legs(dev, dist, rank, world,
                                                       settle_ms=min(args.settle_ms, 150.0))
            except Exception as e:
                log("scaling legs failed:", repr(e))
    if rank == 0:
        if args.legs_out:
            with open(args.legs_out, "w") as f:
                json.dump(result, f)
        line = compact_line(result)
        if len(line) > LINE_BUDGET:  # never let the legs cost the headline its parse
            log(f"compact line {len(line)} chars > {LINE_BUDGET}: dropping the per-leg summary")
            result = {k: v for k, v in result.items() if k not in ("extra", "extra_scaling")}
            line = compact_line(result)
        print(line, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
