"""Worker bodies for the multi-process (gloo) tests; importable by spawned children."""
import os

import numpy as np


def init_gloo(rank, world, port):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def global_average_worker(rank, world, port, out_dir, use_gpu):
    """Each rank owns its column segments of a C12 field; partials from numpy
    (CPU) or the HIP reduction (GPU), combined by fv3net_amd.distributed."""
    import torch

    from fv3net_amd import distributed as D

    dist = init_gloo(rank, world, port)
    rng = np.random.default_rng(0)
    x = rng.normal(280, 20, (6, 12, 12)).astype(np.float32)
    area = rng.uniform(0.5, 1.0, (6, 12, 12)).astype(np.float32)
    segs = D.column_segments(6, 12, rank, world)
    if use_gpu:
        torch.cuda.set_device(0)
        parts = []
        for s in segs:
            xs = torch.from_numpy(x[s.tile, s.y0:s.y1]).cuda()
            a = torch.from_numpy(area[s.tile, s.y0:s.y1]).cuda()
            parts.append(D.area_weighted_partials([xs, xs * 2], a).cpu())
        part = sum(parts[1:], parts[0]) if parts else torch.zeros((2, 2), dtype=torch.float64)
    else:
        part = torch.zeros((2, 2), dtype=torch.float64)
        for s in segs:
            xs = x[s.tile, s.y0:s.y1].astype(np.float64)
            a = area[s.tile, s.y0:s.y1].astype(np.float64)
            part += torch.tensor([[np.sum(a * xs), np.sum(a)], [np.sum(a * xs * 2), np.sum(a)]])
    means = D.global_average(part)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), means)
    dist.barrier()
    dist.destroy_process_group()


def rank_order_worker(rank, world, port, out_dir):
    """Partials chosen so that the summation order changes the result bits."""
    import torch

    from fv3net_amd import distributed as D

    dist = init_gloo(rank, world, port)
    vals = [1e16, 1.0, -1e16, 3.0]
    part = torch.tensor([[vals[rank], 1.0]], dtype=torch.float64)
    total = D.combine_partials(part)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), total.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _lane_sum(v):
    """The kernels' order: lane-strided sequential sums over 64 lanes, then the xor
    butterfly (offsets 32, 16, ..., 1); v is summed along axis 0."""
    lanes = np.zeros((64,) + v.shape[1:])
    for c in range(v.shape[0]):
        lanes[c % 64] = lanes[c % 64] + v[c]
    for o in (32, 16, 8, 4, 2, 1):
        lanes = lanes + lanes[np.arange(64) ^ o]
    return lanes[0]


def fold_rows_np(rows):
    """fv3_fold_rows restated."""
    return _lane_sum(np.asarray(rows))


def _rows_partials_np(x, area):
    """numpy restatement of fv3_area_weighted_row_sums for (rows, row_len) float64
    fields: per row, lane-strided sequential sums over 64 lanes, then the kernel's
    xor butterfly (offsets 32, 16, ..., 1)."""
    return np.array([[_lane_sum(area[r] * x[r]), _lane_sum(area[r])] for r in range(x.shape[0])])


def gather_rows_worker(rank, world, port, out_dir):
    """Each rank owns a row band of a (rows, x) field: its row partials, gathered in
    global row order and folded row by row, must give the world-1 bits."""
    import torch

    from fv3net_amd import distributed as D

    dist = init_gloo(rank, world, port)
    rng = np.random.default_rng(1)
    nrows, nx = 6 * 12, 12
    x = rng.normal(280, 20, (nrows, nx))
    area = rng.uniform(0.5, 1.0, (nrows, nx))
    r0, r1 = D.row_band(nrows, rank, world)
    local = torch.from_numpy(_rows_partials_np(x[r0:r1], area[r0:r1]))
    rows = D.gather_rows(local).numpy()
    total = fold_rows_np(rows)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), np.concatenate([total, rows.reshape(-1)]))
    dist.barrier()
    dist.destroy_process_group()


def sharded_stepper_worker(rank, world, port, out_dir, res, steps, backend="gloo"):
    """The config #4 sharded stepper (workloads.ShardedStepperWorkload) on one GPU per
    rank process (gloo, or nccl = RCCL for a single rank on the box's one GPU, for the
    exchange): global sums and this rank's state band."""
    import torch
    import torch.distributed as tdist

    from fv3net_amd import workloads as W

    if backend == "gloo":
        dist = init_gloo(rank, world, port)
    else:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        tdist.init_process_group(backend, rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        dist = tdist
    torch.cuda.set_device(0)
    wl = W.make_sharded_stepper_workload(res, rank, world, seed=5)
    for _ in range(steps):
        total = wl.step()
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, f"total{rank}.npy"), total.cpu().numpy())
    np.save(os.path.join(out_dir, f"q{rank}.npy"), wl.state["specific_humidity"].cpu().numpy())
    np.save(os.path.join(out_dir, f"rows{rank}.npy"), np.array(wl.rows))
    dist.barrier()
    dist.destroy_process_group()


def count_sums_worker(rank, world, port, out_dir):
    """Integer-valued float64 level counts summed over ranks by one all-reduce
    (distributed.global_count_sums): exact, so every rank and world size agree."""
    import torch

    from fv3net_amd import distributed as D

    dist = init_gloo(rank, world, port)
    counts = np.random.default_rng(7).integers(0, 2 ** 40, (world, 79)).astype(np.float64)
    total = D.global_count_sums(torch.from_numpy(counts[rank]))
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), total.numpy())
    dist.barrier()
    dist.destroy_process_group()


def predict_mappm_worker(rank, world, port, out_dir, res, steps, precision="f32"):
    """north_star's predict + mappm (workloads.PredictMappmWorkload) on this rank's row
    band of one global C<res> state (gloo; ranks share the box's one GPU): the band's
    tendencies and remapped tendencies after ``steps`` steps."""
    import torch

    from fv3net_amd import distributed as D
    from fv3net_amd import workloads as W

    dist = init_gloo(rank, world, port)
    torch.cuda.set_device(0)
    wl = W.make_predict_mappm_workload(res, rank, world, seed=3, precision=precision)
    for _ in range(steps):
        wl.step()
    torch.cuda.synchronize()
    out = np.stack([o.reshape(o.shape[0], -1).cpu().numpy() for o in wl.outputs] +
                   [r.cpu().numpy() for r in wl.remapped])
    np.save(os.path.join(out_dir, f"out{rank}.npy"), out)
    np.save(os.path.join(out_dir, f"rows{rank}.npy"), np.array(D.row_band(6 * res, rank, world)))
    dist.barrier()
    dist.destroy_process_group()
