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
